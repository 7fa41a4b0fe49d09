"""Summarise rocprofv3 --pmc CSVs (tools/pmc_run.sh) per kernel and grid size:
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
