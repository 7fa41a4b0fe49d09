"""Full-size golden proof: the CPU restatement (oracle/, C + OpenMP) proves the
SAME HEIGHT=15-shaped instance bench.py builds on the GPU (bench.Synthetic,
mirrored on the CPU by tests/synth_cpu.py) at n = 2^22, the proof is checked
by the oracle verifier (trapdoor and, with oracle/_ref built, the
reference's blst pairing), and only data is written:

    tests/golden/full_2e22_seed<S>.json : seed, gates, PI, tau, the 2656-byte
        ProofC (hex), the verifier key (hex), and the CPU timings.

Run in the build container (64 GiB, ~30 min on 8 cores):
    python tests/golden/make_golden_full.py [--lg 22] [--seed 1]
The GPU test tests/test_gpu_full.py regenerates the instance on the MI355X,
proves it, and requires the bytes to match.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import pnp_testlib  # noqa: E402,F401  (sys.path)
from pnp import abi  # noqa: E402
from pnp_testlib import oracle, verify, kzg_points, fr_unmont, from_limbs  # noqa: E402
from synth_cpu import SyntheticCPU  # noqa: E402

HEIGHT15_GATES = 3_161_924


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lg", type=int, default=22)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default=None)
    ap.add_argument("--circuit", default="arith", choices=("arith", "merkle"))
    args = ap.parse_args()
    gates = int(HEIGHT15_GATES / (1 << 22) * (1 << args.lg)) if args.lg != 22 else HEIGHT15_GATES
    lib = oracle()
    t0 = time.perf_counter()
    syn = SyntheticCPU(args.lg, gates, args.seed, circuit=args.circuit)
    gates = syn.gates
    t1 = time.perf_counter()
    print(f"instance 2^{args.lg} ({gates} gates): {t1 - t0:.1f} s", flush=True)
    proof = syn.oracle_proof()
    t2 = time.perf_counter()
    print(f"oracle gen_proof: {t2 - t1:.1f} s on {lib.or_num_threads()} threads", flush=True)
    vk = syn.vk()
    t3 = time.perf_counter()
    ok = verify(vk, proof, syn.pis(), syn.tau_mont[0])
    print(f"verifier key {t3 - t2:.1f} s; trapdoor verify: {ok}", flush=True)
    assert ok
    pairing = None
    blst_path = os.path.join(pnp_testlib.REPO, "oracle", "_ref", "libblst_ref.so")
    if os.path.exists(blst_path):
        from test_verifier import _blst, pairing_ok
        rc, pts = kzg_points(vk, proof, syn.pis())
        tau = fr_unmont(from_limbs(syn.tau_mont[0]))
        pairing = rc == 0 and pairing_ok(_blst(), pts[0], pts[1], tau) and pairing_ok(_blst(), pts[2], pts[3], tau)
        print(f"blst pairing verify: {pairing}", flush=True)
        assert pairing
    out = {
        "what": f"oracle (CPU restatement) proof of bench.Synthetic(lg, gates, seed, circuit={args.circuit!r})",
        "circuit": args.circuit, "lg": args.lg, "gates": gates, "seed": args.seed,
        "pi_pos": syn.pi_pos, "pi": syn.pi_canon,
        "tau_mont": [int(v) for v in syn.tau_mont[0]],
        "proof_hex": abi.proof_to_bytes(proof).hex(),
        "vk_hex": vk.tobytes().hex(),
        "verified": {"trapdoor": ok, "blst_pairing": pairing},
        "cpu_seconds": {"instance": round(t1 - t0, 1), "gen_proof": round(t2 - t1, 1),
                        "threads": int(lib.or_num_threads()), "host": "build container"},
    }
    if args.circuit == "merkle":
        out["height"] = syn.height
        out["root"] = hex(syn.root)
    name = (f"merkle_h{args.lg - 7}_seed{args.seed}.json" if args.circuit == "merkle"
            else f"full_2e{args.lg}_seed{args.seed}.json")
    path = args.out or os.path.join(HERE, name)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
