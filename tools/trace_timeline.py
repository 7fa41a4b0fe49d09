"""Per-proof kernel timeline from a rocprofv3 kernel_trace.csv of a bench run:
    python tools/trace_timeline.py run_kernel_trace.csv [proof_index]
Every proof starts with the marker kernel k_proof_begin (csrc/protocol.hip);
a proof spans from its marker to the last kernel before the next marker (the
last proof: to the last kernel of the trace), so setup work before the first
marker (table build, synthetic inputs) is never counted.  Prints the kernel
totals and the GPU idle gaps (host time) of the chosen proof (default: the
last complete one)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
marks = [i for i, e in enumerate(ev) if "k_proof_begin" in e[2]]
if not marks:
    sys.exit("no k_proof_begin markers in the trace (library older than round 2?)")
bounds = [(m, (marks[k + 1] if k + 1 < len(marks) else len(ev))) for k, m in enumerate(marks)]
# the last proof may be cut off by the end of the trace: default to the one before
which = int(sys.argv[2]) if len(sys.argv) > 2 else max(0, len(bounds) - 2)
start, stop = bounds[which]
seg = ev[start:stop]
t0, t1 = seg[0][0], seg[-1][1]
tot = defaultdict(lambda: [0, 0])
gaps, last_end = [], t0
for s, e, n in seg:
    name = n.split("(")[0]
    tot[name][0] += 1
    tot[name][1] += e - s
    if s > last_end:
        gaps.append((s - last_end, name, (s - t0) / 1e6))
    last_end = max(last_end, e)
busy = sum(v[1] for v in tot.values())
print(f"proof {which}: span {(t1 - t0) / 1e6:.2f} ms, kernel busy {busy / 1e6:.2f} ms, "
      f"gaps {sum(g[0] for g in gaps) / 1e6:.2f} ms, kernels {len(seg)}")
for name, (c, ns) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
    if ns > 1e5:
        print(f"  {ns / 1e6:8.3f} ms  {c:4d}x  {name}")
print("largest gaps (us, next kernel, at ms):")
for g, n, at in sorted(gaps, reverse=True)[:8]:
    print(f"  {g / 1e3:8.1f}  {n}  @{at:.2f}")
