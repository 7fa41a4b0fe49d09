"""Per-kernel summary of rocprofv3 --pmc passes (tools/pmc_r02.sh output):
counters summed over the dispatches of a kernel, kernel time from the
dispatch timestamps, and the derived ratios DESIGN.md §5 quotes.

    python tools/pmc_clock.py gpurun_out/r02_pmc > profiles/r02_pmc_clock.txt

Effective clock: GRBM_GUI_ACTIVE is summed over the 8 XCDs
(MI355X_MICROARCH.md, DVFS give-back), so clock = GRBM_GUI_ACTIVE / 8 / time;
SQ_BUSY_CYCLES is summed over the 32 shader engines: clock = it / 32 / time
(each over the dispatch time of its own pass).
"""
import collections
import csv
import glob
import os
import sys


def load(root):
    val = collections.defaultdict(dict)      # kernel -> counter -> sum
    where = collections.defaultdict(dict)    # kernel -> counter -> pass
    ns = collections.defaultdict(lambda: collections.defaultdict(float))   # kernel -> pass -> ns
    disp = collections.defaultdict(lambda: collections.defaultdict(int))
    for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
        p = os.path.basename(os.path.dirname(f))
        seen = set()
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pnp::", "")
            c = r["Counter_Name"]
            val[k][c] = val[k].get(c, 0.0) + float(r["Counter_Value"])
            where[k][c] = p
            if r["Dispatch_Id"] not in seen:
                seen.add(r["Dispatch_Id"])
                ns[k][p] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                disp[k][p] += 1
    return val, where, ns, disp


def main(root):
    val, where, ns, disp = load(root)
    print(f"# per-kernel PMC summary of {root} (sums over dispatches; one bench proof per pass)")
    for k, v in val.items():
        print(f"\n## {k}")
        for p in sorted(ns[k]):
            print(f"  pass {p}: {disp[k][p]} dispatches, {ns[k][p] / 1e6:.3f} ms")
        for c in sorted(v):
            print(f"  {c:28s} {v[c]:.6g}")
        if v.get("SQ_INSTS_VALU") and "SQ_WAVE_CYCLES" in v:
            print(f"  wave_cycles / VALU inst       {v['SQ_WAVE_CYCLES'] / v['SQ_INSTS_VALU']:.3f}")
            for c in ("SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"):
                if c in v:
                    print(f"  {c} / wave_cycles {v[c] / v['SQ_WAVE_CYCLES']:.3f}")
        for c, div in (("SQ_BUSY_CYCLES", 32), ("GRBM_GUI_ACTIVE", 8)):
            if c in v:
                t = ns[k][where[k][c]]
                print(f"  clock from {c:16s}   {v[c] / div / t:.3f} GHz")
        if v.get("SQ_INSTS_LDS"):
            print(f"  LDS bank conflicts / LDS inst {v['SQ_LDS_BANK_CONFLICT'] / v['SQ_INSTS_LDS']:.3f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r02_pmc")
