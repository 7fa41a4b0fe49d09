"""FETCH_SIZE + WRITE_SIZE per k_accumulate29 launch from a tools/pmc_run.sh
output directory -> the JSON bench.py reads for roofline.traffic:
    python tools/pmc_traffic.py gpurun_out/<tag> > profiles/r01_pmc/accumulate_traffic.json"""
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
vals = {"FETCH_SIZE": [], "WRITE_SIZE": []}
for f in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if "k_accumulate29" in r["Kernel_Name"] and r["Counter_Name"] in vals:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]) * 1e3)  # KB -> B
fetch = sum(vals["FETCH_SIZE"]) / max(len(vals["FETCH_SIZE"]), 1)
write = sum(vals["WRITE_SIZE"]) / max(len(vals["WRITE_SIZE"]), 1)
json.dump({
    "kernel": "k_accumulate29",
    "launches": len(vals["FETCH_SIZE"]),
    "fetch_bytes_per_launch": fetch,
    "write_bytes_per_launch": write,
    "bytes_per_launch": fetch + write,
    "note": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate passes over one bench proof "
            "(tools/pmc_run.sh); FETCH_SIZE not doubled: the table gathers are 16-B-per-lane LDS-DMA "
            "loads of 128-B points, not wide coalesced streams (MI355X_MICROARCH.md HBM); algorithmic "
            "bytes per launch = n*(96+32)*MSMs in the batch",
}, sys.stdout, indent=1)
print()
