"""Time of one traced proof during which no VALU-heavy kernel runs (only the
sort, the bucket tail, copies...): the latency-bound share of the span.
    python tools/exposed.py run_kernel_trace.csv [proof_index]"""
import csv
import sys

HEAVY = ("k_accumulate29", "k_ntt_pass", "k_quotient", "k_t_combine", "k_lincomb", "k_perm_numden",
         "k_widgets", "k_horner", "k_eval_partial")
rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]) for r in rows)
marks = [i for i, e in enumerate(ev) if "k_proof_begin" in e[2]]
which = int(sys.argv[2]) if len(sys.argv) > 2 else max(0, len(marks) - 2)
seg = ev[marks[which]:(marks[which + 1] if which + 1 < len(marks) else len(ev))]
t0, t1 = seg[0][0], max(e for _, e, _ in seg)
heavy = sorted((s, e) for s, e, n in seg if any(h in n for h in HEAVY))
cov, cur_s, cur_e = 0, None, None
for s, e in heavy:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            cov += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
if cur_e is not None:
    cov += cur_e - cur_s
span = t1 - t0
print(f"span {span / 1e6:.2f} ms, VALU-heavy kernels cover {cov / 1e6:.2f} ms, exposed {(span - cov) / 1e6:.2f} ms")
# exposed intervals by the kernels running then
expo = {}
pts = sorted(set([t0, t1] + [s for s, _, _ in seg] + [e for _, e, _ in seg]))
hv = heavy
import bisect
for a, b in zip(pts, pts[1:]):
    if b <= a:
        continue
    m = (a + b) / 2
    if any(s <= m < e for s, e in hv):
        continue
    running = [n for s, e, n in seg if s <= m < e]
    key = running[0] if running else "(idle)"
    expo[key] = expo.get(key, 0) + (b - a)
for k, v in sorted(expo.items(), key=lambda kv: -kv[1])[:12]:
    print(f"  {v / 1e6:7.3f} ms  {k}")
# where in the proof (5-ms bins): exposed time per bin
bins = {}
for a, b in zip(pts, pts[1:]):
    if b <= a:
        continue
    m = (a + b) / 2
    if any(s <= m < e for s, e in hv):
        continue
    k = int((m - t0) / 5e6)
    bins[k] = bins.get(k, 0) + (b - a)
print("exposed per 5-ms bin of the proof:", " ".join(f"{5 * k}:{v / 1e6:.2f}" for k, v in sorted(bins.items()) if v > 1e5))
