"""FETCH_SIZE + WRITE_SIZE per k_accumulate29 launch from a tools/gpu.sh traffic
output directory -> the JSON bench.py reads for roofline.traffic:
    python tools/pmc_traffic.py gpurun_out/<tag> > profiles/r02_accumulate_traffic.json
FETCH_SIZE is scaled by the calibration of the gather pattern measured with
tools/ubench_gather.hip (profiles/r02_pmc_gather_calibration.json)."""
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
CAL = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "r02_pmc_gather_calibration.json")
factor = json.load(open(CAL))["factor_true_over_fetch"]
raw = sum(vals["FETCH_SIZE"]) / max(len(vals["FETCH_SIZE"]), 1)
fetch = raw * factor
write = sum(vals["WRITE_SIZE"]) / max(len(vals["WRITE_SIZE"]), 1)
json.dump({
    "kernel": "k_accumulate29",
    "launches": len(vals["FETCH_SIZE"]),
    "fetch_size_bytes_per_launch_raw": raw,
    "fetch_calibration": factor,
    "fetch_bytes_per_launch": fetch,
    "write_bytes_per_launch": write,
    "bytes_per_launch": fetch + write,
    "note": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate passes over one bench proof "
            "(tools/gpu.sh pmc / traffic steps); FETCH_SIZE x the calibration of the same gather pattern on a known byte "
            "count (tools/ubench_gather.hip, MI355X_MICROARCH.md HBM: other access widths are "
            "uncalibrated); expected: one 128-B table line per (point, window) plus the sorted indices",
}, sys.stdout, indent=1)
print()
