"""CPU-baseline scaling: time the C restatement's gen_proof (oracle/, OpenMP)
on bench.Synthetic's instance shape at several domain sizes on ONE host and
fit t = a n^b, so bench.py's bounded CPU sample (2^17) can be extrapolated to
the headline 2^22 with a measured exponent instead of an assumed n log n.

    python tools/cpu_scaling.py --lgs 15 17 19 [--with-golden] > profiles/r02_cpu_scaling.json

--with-golden adds the measured 2^22 point that tests/golden/make_golden_full.py
recorded on the same host (the build container).
"""
import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))

import pnp_testlib  # noqa: E402,F401
from pnp_testlib import oracle  # noqa: E402
from synth_cpu import SyntheticCPU  # noqa: E402

HEIGHT15_GATES = 3_161_924


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lgs", type=int, nargs="+", default=[15, 17, 19])
    ap.add_argument("--with-golden", action="store_true")
    args = ap.parse_args()
    lib = oracle()
    pts = []
    for lg in args.lgs:
        gates = int(HEIGHT15_GATES / (1 << 22) * (1 << lg))
        syn = SyntheticCPU(lg, gates, seed=1)
        t0 = time.perf_counter()
        syn.oracle_proof()
        dt = time.perf_counter() - t0
        pts.append({"lg": lg, "gates": gates, "seconds": round(dt, 3)})
        print(f"2^{lg}: {dt:.2f} s", file=sys.stderr, flush=True)
        del syn
    if args.with_golden:
        with open(os.path.join(REPO, "tests", "golden", "full_2e22_seed1.json")) as f:
            g = json.load(f)
        pts.append({"lg": 22, "gates": g["gates"], "seconds": g["cpu_seconds"]["gen_proof"],
                    "source": "tests/golden/full_2e22_seed1.json"})
    # least squares on log t = log a + b log n
    xs = [p["lg"] * math.log(2) for p in pts]
    ys = [math.log(p["seconds"]) for p in pts]
    mx, my = sum(xs) / len(xs), sum(ys) / len(ys)
    b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    a = math.exp(my - b * mx)
    out = {"what": "C restatement gen_proof seconds vs domain size (instance generation excluded)",
           "threads": int(lib.or_num_threads()), "points": pts,
           "fit": {"model": "t = a * n^b", "exponent": round(b, 4), "a": a,
                   "predicted_2e22_s": round(a * (1 << 22) ** b, 1)}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
