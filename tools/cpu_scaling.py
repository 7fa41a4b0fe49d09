"""CPU-baseline scaling on the GPU box's host: time the C restatement's
gen_proof (oracle/, OpenMP on every host thread) on bench.py's own instance
(bench.Synthetic, generated on the GPU and copied to host memory, generation
not timed) at several domain sizes, check each CPU proof equals the GPU's,
and fit t = a n^b over the measured points.  bench.py's cpu_baseline then
extrapolates its bounded sample with this box-side exponent and reports the
measured full-size (2^22) time beside it.

    python tools/cpu_scaling.py --circuit merkle --lgs 16 17 18 19 20 22 \
        > profiles/r03_cpu_scaling_box.json
"""
import argparse
import ctypes as C
import json
import math
import os
import platform
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import bench  # noqa: E402


def heartbeat(stop):
    """a progress line every minute (a quiet GPU-box command is taken for hung)"""
    t0 = time.perf_counter()
    while not stop.wait(60):
        print(f"  ... {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lgs", type=int, nargs="+", default=[16, 17, 18, 19, 20])
    ap.add_argument("--circuit", default="merkle", choices=("merkle", "arith"))
    args = ap.parse_args()
    import torch
    import pnp
    from pnp import abi
    from pnp_testlib import oracle
    lib = oracle()
    ctx = pnp.Context(0)
    pts = []
    for lg in args.lgs:
        gates = int(bench.HEIGHT15_GATES / (1 << 22) * (1 << lg)) if lg != 22 else bench.HEIGHT15_GATES
        syn = bench.Synthetic(ctx, lg, gates, seed=1, circuit=args.circuit)
        gpu = abi.proof_to_bytes(bench.prove_resident(ctx, syn))
        cs_h, pk_h, ck_h, keep = bench.host_copy(syn)
        del syn
        torch.cuda.empty_cache()
        out = abi.ProofC()
        stop = threading.Event()
        threading.Thread(target=heartbeat, args=(stop,), daemon=True).start()
        t0 = time.perf_counter()
        rc = lib.or_gen_proof(C.byref(cs_h), C.byref(pk_h), C.byref(ck_h), C.byref(out))
        dt = time.perf_counter() - t0
        stop.set()
        same = rc == 0 and abi.proof_to_bytes(out) == gpu
        pts.append({"lg": lg, "gates": int(cs_h.n), "seconds": round(dt, 3), "equals_gpu_proof": same})
        print(f"2^{lg}: {dt:.2f} s, CPU proof == GPU proof: {same}", file=sys.stderr, flush=True)
        del keep
    ctx.close()
    fit_pts = [p for p in pts if p["lg"] <= 20] or pts
    xs = [p["lg"] * math.log(2) for p in fit_pts]
    ys = [math.log(p["seconds"]) for p in fit_pts]
    mx, my = sum(xs) / len(xs), sum(ys) / len(ys)
    b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    a = math.exp(my - b * mx)
    out = {"what": "C restatement gen_proof seconds vs domain size on the GPU box's host "
                   "(bench.Synthetic instance, generation excluded)",
           "circuit": args.circuit, "threads": int(lib.or_num_threads()), "host": platform.node(),
           "cpu": platform.processor() or platform.machine(), "points": pts,
           "fit": {"model": "t = a * n^b over the points up to 2^20", "exponent": round(b, 4), "a": a,
                   "predicted_2e22_s": round(a * (1 << 22) ** b, 1)}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
