"""Per-proof kernel timeline from a rocprofv3 kernel_trace.csv:
    python tools/trace_timeline.py run_kernel_trace.csv [proof_index]
Splits the trace into proofs at the first kernel of each round-1 iNTT burst
(the last `steps` proofs of a bench run), prints per-kernel totals and the GPU
idle gaps (host time) of the chosen proof."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
# proofs start with k_digits? no: find 'k_quotient_' occurrences: one per proof
qi = [i for i, e in enumerate(ev) if e[2].startswith("pnp::k_quotient_")]
which = int(sys.argv[2]) if len(sys.argv) > 2 else -1
q = qi[which]
prev_q = qi[which - 1] if which != 0 and len(qi) > 1 else None
# proof window: from after the previous proof's last kernel (k_lincomb x2 + MSM)... use midpoints
lo = 0 if prev_q is None else prev_q
hi = qi[which + 1] if which + 1 < len(qi) and which != -1 else len(ev)
# refine: start = first kernel after previous quotient whose name is ntt-ish after the last MSM of prev proof
seg = ev[lo:hi]
# locate proof start as the first 'k_dif' after the last 'k_reduce'/'msm' following prev quotient
start = 0
if prev_q is not None:
    last_msm = max(i for i, e in enumerate(seg) if "reduce" in e[2] or "accumulate" in e[2] or "bucket" in e[2] and i < (q - lo))
    # the proof starts after the opening MSM of the previous proof: last msm kernel before the
    # round-1 iNTTs, i.e. the first msm burst after prev quotient ends the previous proof
    k = 0
    bursts = []
    for i, e in enumerate(seg):
        if i >= q - lo:
            break
        if "k_dif" in e[2] and (i == 0 or "k_dif" not in seg[i - 1][2] and "bitrev" not in seg[i - 1][2]):
            bursts.append(i)
    start = bursts[-1] if bursts else 0
    # walk back: the round-1 iNTTs are preceded by memcpy only; proof start = first k_dif of the
    # burst right after the previous proof's final MSM
    msm_after_prev = [i for i, e in enumerate(seg[: q - lo]) if "k_digits" in e[2]]
    # previous proof: quotient, then t commit, then opening commit (2 digit kernels) -> proof start
    # after the 2nd digits burst following prev quotient
    starts = [i for i in bursts if any(j < i for j in msm_after_prev)]
    start = starts[0] if starts else 0
seg = seg[start:]
end_idx = len(seg)
for i, e in enumerate(seg):
    if i > (q - lo - start) and e[2].startswith("pnp::k_dif") and "k_digits" in seg[i - 1][2]:
        end_idx = i
        break
t0 = seg[0][0]
tot = defaultdict(lambda: [0, 0])
gap = 0
last_end = seg[0][0]
gaps = []
for s, e, n in seg:
    name = n.split("(")[0]
    tot[name][0] += 1
    tot[name][1] += e - s
    if s > last_end:
        gaps.append((s - last_end, name, (s - t0) / 1e6))
        gap += s - last_end
    last_end = max(last_end, e)
span = (last_end - t0) / 1e6
busy = sum(v[1] for v in tot.values()) / 1e6
print(f"proof span {span:.2f} ms, kernel busy {busy:.2f} ms, gaps {gap/1e6:.2f} ms, kernels {len(seg)}")
for name, (c, d) in sorted(tot.items(), key=lambda x: -x[1][1]):
    print(f"{d/1e6:9.3f} ms {c:5d}x  {name}")
print("largest gaps (ms, next kernel, at ms):")
for g in sorted(gaps, reverse=True)[:15]:
    print(f"  {g[0]/1e6:8.3f}  {g[1]}  @{g[2]:.1f}")
