"""Summarise rocprofv3 --pmc CSVs (tools/gpu.sh pmc / traffic steps) per kernel and grid size:
    python tools/pmc_summary.py gpurun_out/<tag> > profiles/<name>.txt
FETCH_SIZE / WRITE_SIZE are in KB as reported (gfx950: FETCH_SIZE counts wide
coalesced streaming reads at half their bytes, MI355X_MICROARCH.md HBM)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        key = (name, int(r["Grid_Size"]), int(r["VGPR_Count"]), int(r["LDS_Block_Size"]))
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        acc[key]["_dur_ns"].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
print(f"{'kernel':32s} {'grid':>9s} {'vgpr':>4s} {'n':>4s} {'dur_us':>9s} {'FETCH_MB':>9s} "
      f"{'WRITE_MB':>9s} {'valu/wave':>9s} {'active%':>7s} {'wait%':>6s} {'instwait%':>9s}")
for key in sorted(acc, key=lambda k: -sum(acc[k]["_dur_ns"])):
    d = acc[key]
    mean = lambda c: sum(d[c]) / len(d[c]) if d.get(c) else float("nan")
    n = max(len(d.get("FETCH_SIZE", [])), len(d.get("SQ_WAVES", [])), 1)
    wc = mean("SQ_WAVE_CYCLES")
    print(f"{key[0]:32s} {key[1]:9d} {key[2]:4d} {n:4d} {mean('_dur_ns') / 1e3:9.1f} "
          f"{mean('FETCH_SIZE') / 1e3:9.1f} {mean('WRITE_SIZE') / 1e3:9.1f} "
          f"{mean('SQ_INSTS_VALU') / max(mean('SQ_WAVES'), 1):9.0f} "
          f"{100 * mean('SQ_ACTIVE_INST_ANY') / wc:7.1f} {100 * mean('SQ_WAIT_ANY') / wc:6.1f} "
          f"{100 * mean('SQ_WAIT_INST_ANY') / wc:9.1f}")

# k_accumulate29: the mixed additions the counters allow per launch.  The
# static model of the compiled kernel (tools/isa_model.py) issues ~5,154 VALU
# wave-instructions per 64 lane-additions on its longest path; SQ_INSTS_VALU
# also counts the non-addition work (the binary search, staging, stores).  With
# a bench JSON as the second argument the measured VALU per device-counted
# addition (roofline.madds_per_proof) is printed beside it: a count the
# counters cannot have issued would show as far fewer VALU per addition.
VALU_PER_MADD = 5154
rows = [(k, acc[k]) for k in acc if k[0].endswith("k_accumulate29") and acc[k].get("SQ_INSTS_VALU")]
if rows:
    tot_m = tot_ns = tot_n = 0
    print()
    print(f"{'k_accumulate29 grid':>20s} {'n':>3s} {'dur_us':>9s} {'VALU_G/launch':>13s} {'madds_mdl_M':>11s}")
    for k, d in sorted(rows, key=lambda r: -r[0][1]):
        v = [x for x in d["SQ_INSTS_VALU"]]
        n = len(v)
        m = sum(v) / n * 64 / VALU_PER_MADD
        dur = sum(d["_dur_ns"]) / len(d["_dur_ns"])
        tot_m += m * n
        tot_ns += dur * n
        tot_n += n
        print(f"{k[1]:20d} {n:3d} {dur / 1e3:9.1f} {sum(v) / n / 1e9:13.3f} {m / 1e6:11.2f}")
    print(f"all launches: {tot_n}, madds at the model VALU/addition {tot_m / 1e6:.1f} M, {tot_m / (tot_ns / 1e9) / 1e9:.3f} G madd/s "
          f"over their summed duration")
    if len(sys.argv) > 2:
        import json
        with open(sys.argv[2]) as f:
            counted = json.loads(f.read().strip().splitlines()[-1])["roofline"]["madds_per_proof"]
        valu = sum(sum(d["SQ_INSTS_VALU"]) for _, d in rows)
        print(f"device-counted madds per proof {counted / 1e6:.1f} M (bench): {valu * 64 / counted:.0f} VALU "
              f"lane-instructions per counted madd vs {VALU_PER_MADD} in the static model")
