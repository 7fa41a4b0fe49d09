"""Time the first proofs after a key load at 2^LG (default 22): the first
builds the folded SRS table and, with PNP_DEFER_TABLES=0, the Lagrange basis
and the copy-group tables; by default it goes without them and they build in
the background (context.h), so the next proofs run beside that build; then
the time until it is done (pnp_sync) and a proof with the tables.  Prints
one JSON line.
    python tools/first_proof.py [LG]"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "zprize23-gpu-submission_amd"))


def main():
    import pnp
    from pnp import abi
    from bench import Synthetic
    lg = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    ctx = pnp.Context(0)
    try:
        syn = Synthetic(ctx, lg, 0, seed=1, circuit="merkle")
        ctx.sync()
        t0 = time.perf_counter()
        ctx.load_prover_key(syn.pk, syn.n, device_ptrs=True)
        ctx.load_commit_key(syn.ck, syn.n, device_ptrs=True)
        ctx.sync()
        t_load = time.perf_counter() - t0
        times, proofs = [], []
        for _ in range(3):  # (pnp_prove returns with its proof done; no sync: that would wait for the build)
            t0 = time.perf_counter()
            proofs.append(abi.proof_to_bytes(ctx.prove(syn.cs, device_ptrs=True)))
            times.append(round(time.perf_counter() - t0, 4))
        t0 = time.perf_counter()
        ctx.sync()
        build_left = round(time.perf_counter() - t0, 4)
        t0 = time.perf_counter()
        proofs.append(abi.proof_to_bytes(ctx.prove(syn.cs, device_ptrs=True)))
        after = round(time.perf_counter() - t0, 4)
        print(json.dumps({"lg": lg, "defer_tables": os.environ.get("PNP_DEFER_TABLES", "default (on at world 1)"),
                          "key_load_s": round(t_load, 4), "proof_s": times,
                          "background_build_left_s": build_left, "proof_after_build_s": after,
                          "proofs_identical": all(p == proofs[0] for p in proofs)}))
    finally:
        ctx.close()


if __name__ == "__main__":
    main()
