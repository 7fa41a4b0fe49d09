"""Folded-MSM window sweep at one rank's point range: time pnp_commit_ck (one
MSM, the resident folded table) for 2^lg points and window bits c, as a rank
of an N-GPU proof at n = 2^22 sees it (2^21 / 2^20 / 2^19 points for N = 2 /
4 / 8).  Prints one JSON line per (lg, c).
    python tools/msm_c_sweep.py [lg ...]
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "zprize23-gpu-submission_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    import torch
    import pnp
    from pnp import abi
    from gpu_util import empty_dev, from_dev
    lgs = [int(a) for a in sys.argv[1:]] or [19, 20, 21]
    for lg in lgs:
        n = 1 << lg
        for c in ([int(os.environ["SWEEP_C"])] if os.environ.get("SWEEP_C") else range(max(14, lg - 5), 21)):
            os.environ["PNP_FOLD_C"] = str(c)
            ctx = pnp.Context(0)
            srs = empty_dev(n, 12)
            tau = empty_dev(1)
            ctx.random_fr(tau.data_ptr(), 1, 77)
            ctx.sync()
            ctx.srs(srs.data_ptr(), n, [int(v) for v in from_dev(tau)[0]])
            ctx.sync()
            ck = abi.CommitKeyC(powers_of_g=abi.ptr(srs.data_ptr()), powers_of_gamma_g=abi.ptr(srs.data_ptr()))
            ctx.load_commit_key(ck, n, device_ptrs=True)
            sc = empty_dev(n)
            ctx.random_fr(sc.data_ptr(), n, 5)
            ctx.sync()
            ctx.commit_ck(sc.data_ptr(), n)  # warm-up
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                ctx.commit_ck(sc.data_ptr(), n)
                ts.append(time.perf_counter() - t0)
            ctx.kernel_timing(True)
            ctx.commit_ck(sc.data_ptr(), n)
            acc_ms, _ = ctx.kernel_stats("msm_accumulate")
            fb = ctx.kernel_bytes("msm_exact_fallback")
            redo = ctx.kernel_bytes("msm_redo_lanes")
            ctx.kernel_timing(False)
            print(json.dumps({"lg": lg, "c": c, "ms_min": round(1e3 * min(ts), 3),
                              "ms_med": round(1e3 * sorted(ts)[2], 3), "accumulate_ms": round(acc_ms, 3),
                              "exact_fallbacks": fb, "redo_lanes": redo}), flush=True)
            ctx.close()
            del srs, sc, tau
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
