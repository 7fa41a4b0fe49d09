"""Full-size parity (BASELINE configs 3 and 4, n = 2^22) on the MI355X.

  * the production folded c = 20 MSM (pnp_commit_ck) on 2^22 points against
    the CPU restatement's Pippenger (oracle/g1.c) on the box's host cores,
    with random scalars and with the degenerate cases (zero and r-1 scalars,
    repeated bases, clustered scalars -> ~10^5-entry buckets);
  * the HEIGHT=15 proof of bench.py's own instance (bench.Synthetic, seed 1,
    3,161,924 gates) byte-identical to the golden ProofC the CPU restatement
    produced for the same instance in the build container
    (tests/golden/make_golden_full.py -> full_2e22_seed1.json), and accepted
    by the restated verifier with the golden verifier key;
  * GPU instance generation == CPU instance generation (tests/synth_cpu.py)
    at a small size, proofs byte-identical."""
import json
import os
import sys

import numpy as np
import pytest

from gpu_util import from_dev, empty_dev, to_dev
from pnp_testlib import REPO, oracle, vp, fr_mont, to_limbs, R_MOD, verify

pytestmark = pytest.mark.gpu
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden", "full_2e22_seed1.json")
GOLDEN_MERKLE = os.path.join(REPO, "tests", "golden", "merkle_h15_seed1.json")
N22 = 1 << 22


def _ck(addr):
    from pnp import abi
    return abi.CommitKeyC(powers_of_g=abi.ptr(addr), powers_of_gamma_g=abi.ptr(addr))


@pytest.fixture(scope="module")
def big():
    """2^22 SRS points ([tau^i] G generated on the GPU; the generator is
    pinned against or_srs by test_gpu_ops) and a context whose commit key is
    that SRS (folded c = 20 table, as for every gen_proof commitment)."""
    import pnp
    ctx = pnp.Context(0)
    srs = empty_dev(N22, 12)
    tau = empty_dev(1)
    ctx.random_fr(tau.data_ptr(), 1, 4242)
    ctx.sync()
    ctx.srs(srs.data_ptr(), N22, [int(v) for v in from_dev(tau)[0]])
    ctx.sync()
    pts = from_dev(srs, 12).copy()
    yield ctx, srs, pts
    ctx.close()


def _check(ctx, pts_dev_addr, pts, sc):
    exp = np.zeros(12, dtype=np.uint64)
    oracle().or_commit(vp(pts), vp(np.ascontiguousarray(sc)), len(pts), vp(exp))
    ctx.load_commit_key(_ck(pts_dev_addr), len(pts), device_ptrs=True)
    d = to_dev(sc)
    c = ctx.commit_ck(d.data_ptr(), len(pts))
    got = np.array(list(c.x) + list(c.y), dtype=np.uint64)
    assert (got == exp).all()


def test_msm_2e22_random_vs_oracle(big):
    ctx, srs, pts = big
    sc = empty_dev(N22)
    ctx.random_fr(sc.data_ptr(), N22, 99)
    ctx.sync()
    h = from_dev(sc).copy()
    h[::7] = 0
    _check(ctx, srs.data_ptr(), pts, h)


@pytest.mark.parametrize("lg", [18, 19])
def test_msm_rank_range_vs_oracle(big, lg):
    """The folded MSM at one rank's point range of a 16 / 8-GPU proof at 2^22
    (2^18 / 2^19 points: c = 15 / 20, msm_cfg) vs the oracle."""
    ctx, srs, pts = big
    m = 1 << lg
    sc = empty_dev(m)
    ctx.random_fr(sc.data_ptr(), m, 1000 + lg)
    ctx.sync()
    h = from_dev(sc).copy()
    h[::5] = 0
    _check(ctx, srs.data_ptr(), np.ascontiguousarray(pts[:m]), h)


def test_msm_2e22_degenerate_vs_oracle(big):
    """Repeated bases with equal scalars (equal points inside a bucket piece:
    the exact redo path), r-1, zeros, and ~10^5-entry buckets from a handful
    of distinct scalars, through the same 2^22 folded MSM."""
    ctx, srs, pts = big
    rng = np.random.default_rng(3)
    pts2 = pts.copy()
    pts2[1000:1400] = pts2[17]
    vals = np.array([to_limbs(fr_mont(v), 4) for v in
                     (R_MOD - 1, 1, 2, 12345678901234567890, R_MOD - 2)], dtype=np.uint64)
    sc = np.ascontiguousarray(vals[rng.integers(0, len(vals), size=N22)])
    sc[1000:1400] = sc[17]
    sc[::13] = 0
    d = to_dev(pts2)
    _check(ctx, d.data_ptr(), pts2, sc)


def test_synthetic_gpu_equals_cpu_small():
    """bench.Synthetic on the GPU and tests/synth_cpu.SyntheticCPU build the
    same instance; their proofs (GPU v2 resident path vs CPU restatement) are
    byte-identical and verify."""
    import pnp
    from pnp import abi
    from bench import Synthetic
    from synth_cpu import SyntheticCPU
    lg, gates, seed = 10, 1000, 3
    cpu = SyntheticCPU(lg, gates, seed)
    exp = cpu.oracle_proof()
    ctx = pnp.Context(0)
    try:
        syn = Synthetic(ctx, lg, gates, seed=seed)
        ctx.load_prover_key(syn.pk, syn.n, device_ptrs=True)
        ctx.load_commit_key(syn.ck, syn.n, device_ptrs=True)
        got = ctx.prove(syn.cs, device_ptrs=True)
        assert abi.proof_to_bytes(got) == abi.proof_to_bytes(exp)
        assert verify(cpu.vk(), got, cpu.pis(), cpu.tau_mont[0])
    finally:
        ctx.close()


def test_synthetic_merkle_gpu_equals_cpu_small():
    """bench.Synthetic(circuit="merkle") on the GPU (pnp_synth_merkle) and
    SyntheticCPU(circuit="merkle") (or_synth_merkle) at HEIGHT 5 (2^12): the
    same circuit, witness, root and key; proofs byte-identical, verified."""
    import pnp
    from pnp import abi
    from bench import Synthetic
    from synth_cpu import SyntheticCPU
    lg, seed = 12, 6
    cpu = SyntheticCPU(lg, 0, seed, circuit="merkle")
    exp = cpu.oracle_proof()
    ctx = pnp.Context(0)
    try:
        syn = Synthetic(ctx, lg, 0, seed=seed, circuit="merkle")
        assert (syn.gates, syn.height) == (cpu.gates, 5)
        assert list(syn.pi) == [int(v) for v in cpu.pi_canon]
        for w in ("w_l", "w_r", "w_o", "w_4"):
            assert np.array_equal(syn.keep[w].cpu().numpy().view(np.uint64), cpu.arrays[w]), w
        ctx.load_prover_key(syn.pk, syn.n, device_ptrs=True)
        ctx.load_commit_key(syn.ck, syn.n, device_ptrs=True)
        got = ctx.prove(syn.cs, device_ptrs=True)
        assert abi.proof_to_bytes(got) == abi.proof_to_bytes(exp)
        assert verify(cpu.vk(), got, cpu.pis(), cpu.tau_mont[0])
    finally:
        ctx.close()


def _golden_case(path, circuit):
    import pnp
    from pnp import abi
    from bench import Synthetic
    with open(path) as f:
        g = json.load(f)
    assert g.get("circuit", "arith") == circuit
    ctx = pnp.Context(0)
    try:
        syn = Synthetic(ctx, g["lg"], g["gates"], seed=g["seed"], circuit=circuit)
        assert syn.gates == g["gates"]
        ctx.load_prover_key(syn.pk, syn.n, device_ptrs=True)
        ctx.load_commit_key(syn.ck, syn.n, device_ptrs=True)
        got = ctx.prove(syn.cs, device_ptrs=True)
        assert abi.proof_to_bytes(got).hex() == g["proof_hex"]
        vk = np.frombuffer(bytes.fromhex(g["vk_hex"]), dtype=np.uint64).copy()
        pi = sum(int(v) << (64 * k) for k, v in enumerate(g["pi"]))
        assert verify(vk, got, [(g["pi_pos"], pi)], np.array(g["tau_mont"], dtype=np.uint64))
    finally:
        ctx.close()


@pytest.mark.skipif(not os.path.exists(GOLDEN), reason="golden 2^22 proof not generated")
def test_height15_proof_matches_golden():
    """The round-1 stand-in (random satisfying arithmetic circuit, 3,161,924 gates)."""
    _golden_case(GOLDEN, "arith")


@pytest.mark.skipif(not os.path.exists(GOLDEN_MERKLE), reason="golden HEIGHT=15 Merkle proof not generated")
def test_height15_merkle_proof_matches_golden():
    """The bench's default input: the reference's HEIGHT=15 Poseidon Merkle
    circuit (pnp_synth_merkle, seed 1), byte-identical to the ProofC the CPU
    restatement produced for the same instance (or_synth_merkle,
    tests/golden/make_golden_full.py --circuit merkle) and accepted by the
    restated verifier with the golden verifier key."""
    _golden_case(GOLDEN_MERKLE, "merkle")
