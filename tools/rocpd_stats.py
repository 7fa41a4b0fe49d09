"""Kernel stats CSV from a rocprofv3 rocpd database (the `top_kernels` view):
    python tools/rocpd_stats.py run_results.db > profiles/<name>.csv
Columns: name, calls, total_us, avg_us, percent (durations in microseconds)."""
import csv
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
w = csv.writer(sys.stdout)
w.writerow(["name", "calls", "total_us", "avg_us", "percent"])
for name, calls, total, avg, pct in db.execute(
        "select name, total_calls, total_duration, average, percentage from top_kernels"):
    w.writerow([name, calls, round(total, 3), round(avg, 3), round(pct, 3)])
