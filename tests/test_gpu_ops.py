"""GPU parity of the operator API against the CPU restatement (oracle/).

Every comparison is bit-exact on Montgomery limbs / affine coordinates.
Sizes reach BASELINE config 2 (NTT 2^20) and MSM 2^16 here; the full 2^22
MSM is compared with the oracle directly in tests/test_gpu_full.py.
"""
import ctypes as C
import os

import numpy as np
import pytest

from pnp_testlib import REPO, oracle, vp, rand_fr_mont_arr, from_limbs, R_MOD, fr_mont
from gpu_util import to_dev, from_dev, empty_dev

pytestmark = pytest.mark.gpu

GOLD = np.load(os.path.join(REPO, "tests", "golden", "golden.npz"))


@pytest.fixture(scope="module")
def ctx():
    import pnp
    c = pnp.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("lg", [1, 3, 5, 9, 10, 11, 13, 16, 20])
def test_ntt_vs_oracle(ctx, lg):
    rng = np.random.default_rng(100 + lg)
    x = rand_fr_mont_arr(rng, 1 << lg)
    lib = oracle()
    for inverse, coset in [(0, 0), (1, 0), (0, 1), (1, 1)]:
        exp = x.copy()
        lib.or_ntt(vp(exp), lg, inverse, coset)
        d = to_dev(x)
        ctx.ntt(d.data_ptr(), lg, bool(inverse), bool(coset))
        got = from_dev(d)
        assert (got == exp).all(), (lg, inverse, coset)


@pytest.mark.parametrize("lg", [1, 2, 3, 5, 7])
def test_ntt_golden(ctx, lg):
    x = GOLD[f"ntt{lg}_in"]
    for inverse, coset, key in [(0, 0, "fwd"), (1, 0, "inv"), (0, 1, "coset_fwd"), (1, 1, "coset_inv")]:
        d = to_dev(x)
        ctx.ntt(d.data_ptr(), lg, bool(inverse), bool(coset))
        assert (from_dev(d) == GOLD[f"ntt{lg}_{key}"]).all(), key


@pytest.mark.parametrize("lg", [3, 8, 12])
def test_coset_lde8(ctx, lg):
    rng = np.random.default_rng(7 + lg)
    x = rand_fr_mont_arr(rng, 1 << lg)
    exp = np.zeros((8 << lg, 4), dtype=np.uint64)
    oracle().or_coset_lde8(vp(x), vp(exp), lg)
    src = to_dev(x)
    dst = empty_dev(8 << lg)
    ctx.coset_lde8(src.data_ptr(), dst.data_ptr(), lg)
    assert (from_dev(dst) == exp).all()


def _commit_dev(ctx, pts, sc_mont):
    dp, ds = to_dev(pts), to_dev(sc_mont)
    c = ctx.commit(dp.data_ptr(), ds.data_ptr(), len(pts))
    return np.array(list(c.x) + list(c.y), dtype=np.uint64)


def _commit_ck(ctx, pts, sc_mont):
    """Commitment through the resident commit key: the folded fixed-base
    layout gen_proof uses (table of 2^(c k) multiples built on first use)."""
    from pnp import abi
    dp, ds = to_dev(pts), to_dev(sc_mont)
    ck = abi.CommitKeyC(powers_of_g=abi.ptr(dp.data_ptr()), powers_of_gamma_g=abi.ptr(dp.data_ptr()))
    ctx.load_commit_key(ck, len(pts), device_ptrs=True)
    c = ctx.commit_ck(ds.data_ptr(), len(pts))
    return np.array(list(c.x) + list(c.y), dtype=np.uint64)


@pytest.mark.parametrize("n", [1, 2, 3, 17, 64, 257, 1024])
def test_msm_golden(ctx, n):
    pts = GOLD[f"msm{n}_points"]
    sc = GOLD[f"msm{n}_scalars"].copy()
    oracle().or_fr_vec_to_mont(vp(sc), n)
    assert (_commit_dev(ctx, pts, sc) == GOLD[f"msm{n}_result"]).all()
    assert (_commit_ck(ctx, pts, sc) == GOLD[f"msm{n}_result"]).all()


@pytest.mark.parametrize("n", [5000, 1 << 14, 1 << 16])
def test_msm_vs_oracle(ctx, n):
    rng = np.random.default_rng(n)
    lib = oracle()
    tau = rand_fr_mont_arr(rng, 1)
    pts = np.zeros((n, 12), dtype=np.uint64)
    lib.or_srs(vp(pts), n, vp(tau))
    sc = rand_fr_mont_arr(rng, n)
    sc[::7] = 0  # zero digits / zero scalars
    exp = np.zeros(12, dtype=np.uint64)
    lib.or_commit(vp(pts), vp(sc), n, vp(exp))
    assert (_commit_dev(ctx, pts, sc) == exp).all()
    assert (_commit_ck(ctx, pts, sc) == exp).all()


@pytest.mark.parametrize("c", [18, 20])
def test_msm_folded_wide_windows(c, monkeypatch):
    """The folded fixed-base layout with the wide windows used at 2^22 (and the
    running-sum tree leaves), forced on a small MSM (PNP_FOLD_C)."""
    import pnp
    monkeypatch.setenv("PNP_FOLD_C", str(c))
    ctx = pnp.Context(0)
    try:
        n = 5000
        rng = np.random.default_rng(c)
        lib = oracle()
        tau = rand_fr_mont_arr(rng, 1)
        pts = np.zeros((n, 12), dtype=np.uint64)
        lib.or_srs(vp(pts), n, vp(tau))
        pts[100:110] = pts[7]  # repeated bases: degenerate pieces -> exact redo
        sc = rand_fr_mont_arr(rng, n)
        sc[::5] = 0
        sc[100:110] = sc[7]
        exp = np.zeros(12, dtype=np.uint64)
        lib.or_commit(vp(pts), vp(sc), n, vp(exp))
        assert (_commit_ck(ctx, pts, sc) == exp).all()
    finally:
        ctx.close()


def test_msm_folded_multi_tile_bins(monkeypatch):
    """Buckets far larger than one k_fine_sort LDS tile (TILE_F = 8192
    entries) and than one accumulate lane's segment: every scalar is one of
    three values, so each window sends ~n/3 = 10000 entries to ONE bucket
    (coarse bin): the multi-tile cursor path of the fine sort and the
    many-piece merge run (at 2^22 each bin holds ~100K entries)."""
    import pnp
    monkeypatch.setenv("PNP_FOLD_C", "20")
    ctx = pnp.Context(0)
    try:
        n = 30000
        rng = np.random.default_rng(77)
        lib = oracle()
        tau = rand_fr_mont_arr(rng, 1)
        pts = np.zeros((n, 12), dtype=np.uint64)
        lib.or_srs(vp(pts), n, vp(tau))
        vals = rand_fr_mont_arr(rng, 3)
        sc = np.ascontiguousarray(vals[rng.integers(0, 3, size=n)])
        exp = np.zeros(12, dtype=np.uint64)
        lib.or_commit(vp(pts), vp(sc), n, vp(exp))
        assert (_commit_ck(ctx, pts, sc) == exp).all()
    finally:
        ctx.close()


def test_msm_edge_cases(ctx):
    lib = oracle()
    rng = np.random.default_rng(5)
    n = 300
    tau = rand_fr_mont_arr(rng, 1)
    pts = np.zeros((n, 12), dtype=np.uint64)
    lib.or_srs(vp(pts), n, vp(tau))
    pts[10:20] = pts[5]  # repeated bases -> doubling inside buckets
    cases = {
        "zeros": np.zeros((n, 4), dtype=np.uint64),
        "minus_one": np.tile(np.array([(fr_mont(R_MOD - 1) >> (64 * i)) & (2**64 - 1) for i in range(4)],
                                      dtype=np.uint64), (n, 1)),
        "random": rand_fr_mont_arr(rng, n),
    }
    one = np.array([(fr_mont(1) >> (64 * i)) & (2**64 - 1) for i in range(4)], dtype=np.uint64)
    cases["ones"] = np.tile(one, (n, 1))
    # P_i + (-P_i): scalars s and r - s on the same base
    pair = rand_fr_mont_arr(rng, n)
    for i in range(0, n - 1, 2):
        pts[i + 1] = pts[i]
        v = (R_MOD - from_limbs(pair[i])) % R_MOD
        pair[i + 1] = [(v >> (64 * k)) & (2**64 - 1) for k in range(4)]
    cases["cancel"] = pair
    for name, sc in cases.items():
        exp = np.zeros(12, dtype=np.uint64)
        lib.or_commit(vp(pts), vp(sc), n, vp(exp))
        assert (_commit_dev(ctx, pts, sc) == exp).all(), name
        assert (_commit_ck(ctx, pts, sc) == exp).all(), name


@pytest.mark.parametrize("n", [1, 31, 32, 33, 1000, 1 << 16])
def test_scans_vs_oracle(ctx, n):
    rng = np.random.default_rng(n + 11)
    lib = oracle()
    x = rand_fr_mont_arr(rng, n)
    z = rand_fr_mont_arr(rng, 1)[0]
    # prefix product
    exp = x.copy()
    lib.or_prefix_product(vp(exp), n)
    d = to_dev(x)
    ctx.prefix_product(d.data_ptr(), n)
    assert (from_dev(d) == exp).all()
    # division by (X - z)
    exp = x.copy()
    lib.or_poly_div_linear(vp(exp), n, vp(z))
    d = to_dev(x)
    ctx.poly_div_linear(d.data_ptr(), n, [int(v) for v in z])
    assert (from_dev(d) == exp).all()
    # evaluation
    e = np.zeros(4, dtype=np.uint64)
    lib.or_poly_eval(vp(x), n, vp(z), vp(e))
    d = to_dev(x)
    assert ctx.poly_eval(d.data_ptr(), n, [int(v) for v in z]) == [int(v) for v in e]
    # batch inverse (with zeros)
    y = x.copy()
    y[::5] = 0
    exp = y.copy()
    lib.or_batch_inverse(vp(exp), n)
    d = to_dev(y)
    ctx.batch_inverse(d.data_ptr(), n)
    assert (from_dev(d) == exp).all()


def test_batch_inverse_large(ctx):
    n = (1 << 20) + 77
    rng = np.random.default_rng(3)
    x = rand_fr_mont_arr(rng, n)
    exp = x.copy()
    oracle().or_batch_inverse(vp(exp), n)
    d = to_dev(x)
    ctx.batch_inverse(d.data_ptr(), n)
    assert (from_dev(d) == exp).all()


def test_synth_srs_and_coset_consts(ctx):
    """The bench's on-GPU input generators match the CPU restatement."""
    import torch
    lib = oracle()
    rng = np.random.default_rng(77)
    n = 257
    tau = rand_fr_mont_arr(rng, 1)
    exp = np.zeros((n, 12), dtype=np.uint64)
    lib.or_srs(vp(exp), n, vp(tau))
    d = empty_dev(n, 12)
    ctx.srs(d.data_ptr(), n, [int(v) for v in tau[0]])
    assert (from_dev(d, 12) == exp).all()
    from pnp_testlib import Inputs
    inp = Inputs(6, 1)
    vh, x = empty_dev(8 << 6), empty_dev(8 << 6)
    ctx.coset_consts(vh.data_ptr(), x.data_ptr(), 6)
    assert (from_dev(vh) == inp.arrays["v_h_coset_8n"]).all()
    assert (from_dev(x) == inp.arrays["linear_evaluations"]).all()
    r = empty_dev(4096)
    ctx.random_fr(r.data_ptr(), 4096, 5)
    vals = from_dev(r)
    assert all(from_limbs(v) < R_MOD for v in vals[:256])
    assert len({tuple(v) for v in vals}) == 4096


@pytest.mark.parametrize("c", [13, 20])
def test_msm_folded_equal_pieces_exact_fallback(c, monkeypatch):
    """Every point the same P and every scalar the same s: each window puts
    all n entries into one bucket, split across many accumulate lanes whose
    pieces are equal multiples of P, so the radix-2^29 merge meets equal
    operands (an exceptional addition, ec29.cuh) and the group must take the
    exact 32-bit fallback (reduce_group_exact); result n s P vs the oracle."""
    import pnp
    monkeypatch.setenv("PNP_FOLD_C", str(c))
    ctx = pnp.Context(0)
    try:
        n = 6000
        rng = np.random.default_rng(c + 1)
        lib = oracle()
        tau = rand_fr_mont_arr(rng, 1)
        pts = np.zeros((n, 12), dtype=np.uint64)
        lib.or_srs(vp(pts), 2, vp(tau))
        pts[:] = pts[1]
        sc = rand_fr_mont_arr(rng, 1).repeat(n, axis=0)
        exp = np.zeros(12, dtype=np.uint64)
        lib.or_commit(vp(pts), vp(sc), n, vp(exp))
        ctx.kernel_timing(True)
        assert (_commit_ck(ctx, pts, sc) == exp).all()
        assert ctx.kernel_bytes("msm_exact_fallback") >= 1  # the fallback really ran
        ctx.kernel_timing(False)
    finally:
        ctx.close()


def test_commit_key_strided_ark_layout():
    """pnp_load_commit_key_strided: the SRS handed over in arkworks' G1Affine
    memory layout (104-byte stride, x / y / infinity, garbage padding) gives
    the same commitments as the packed CommitKeyC, host and device pointers;
    a point flagged infinity is refused."""
    import numpy as np
    import pnp
    from pnp import abi
    from gpu_util import to_dev, empty_dev
    from pnp_testlib import oracle, vp
    n = 1 << 12
    tau = np.array([[123456789, 5, 0, 7]], dtype=np.uint64)
    srs = np.zeros((n, 12), dtype=np.uint64)
    oracle().or_srs(vp(srs), n, vp(tau))
    rng = np.random.default_rng(5)
    ark = rng.integers(0, 256, size=(n, 104), dtype=np.uint8)  # padding bytes are garbage
    ark[:, 0:96] = srs.view(np.uint8).reshape(n, 96)
    ark[:, 96] = 0
    ctx = pnp.Context(0)
    try:
        sc = empty_dev(n)
        ctx.random_fr(sc.data_ptr(), n, 77)
        ctx.sync()
        ctx.load_commit_key(abi.CommitKeyC(powers_of_g=abi.ptr(srs.ctypes.data),
                                           powers_of_gamma_g=abi.ptr(srs.ctypes.data)), n, device_ptrs=False)
        exp = ctx.commit_ck(sc.data_ptr(), n)
        ctx.load_commit_key_strided(ark.ctypes.data, n)
        got = ctx.commit_ck(sc.data_ptr(), n)
        assert list(got.x) == list(exp.x) and list(got.y) == list(exp.y)
        d = to_dev(ark.view(np.uint64).reshape(n, 13))
        ctx.load_commit_key_strided(d.data_ptr(), n, device_ptrs=True)
        got = ctx.commit_ck(sc.data_ptr(), n)
        assert list(got.x) == list(exp.x) and list(got.y) == list(exp.y)
        ark[77, 96] = 1
        with pytest.raises(pnp.PnpError, match="infinity"):
            ctx.load_commit_key_strided(ark.ctypes.data, n)
        bad = abi.AffineLayout(stride=100, x_off=0, y_off=48, inf_off=96)
        with pytest.raises(pnp.PnpError, match="PNP_E_ARG"):
            ctx.load_commit_key_strided(ark.ctypes.data, n, layout=bad)
    finally:
        ctx.close()


def test_proof_infinity_mask_of_gpu_proof():
    """The mask of a GPU proof of a Merkle-class circuit: f, h1, h2, t7, t8 at
    infinity (the flags merkle-tree/src/main.rs:112-123 hard-codes), nothing
    else; with live lookups f / h1 / h2 are finite."""
    import pnp
    from pnp_testlib import Inputs
    inp = Inputs(8, 2)
    p = pnp.load().gen_proof(inp.circuit, inp.pk, inp.ck)
    flags = pnp.infinity_flags(p)
    assert sorted(k for k, v in flags.items() if v) == ["f_comm", "h_1_comm", "h_2_comm", "t_7_comm", "t_8_comm"]
    inp2 = Inputs(8, 47, lookup_rows=17)
    ctx = pnp.Context(0)
    try:
        ctx.load_prover_key(inp2.pk, inp2.n, device_ptrs=False)
        ctx.load_commit_key(inp2.ck, inp2.n, device_ptrs=False)
        flags = pnp.infinity_flags(ctx.prove(inp2.circuit, device_ptrs=False))
        assert not flags["f_comm"] and not flags["h_1_comm"] and not flags["h_2_comm"]
    finally:
        ctx.close()


# ---- small-n matrix: every MSM entry point at the sizes
# where the per-window layout has more virtual windows (B W = 64 at n = 1,
# c = 4) than the 16 per-MSM segment slots of KeyRows — the r03v illegal
# memory access ("Fault record") — and the segmented copy-group
# batch at B = 1 and B = 4, all against the oracle's Pippenger (oracle/g1.c).
def _srs_host(n, seed):
    rng = np.random.default_rng(seed)
    tau = rand_fr_mont_arr(rng, 1)
    pts = np.zeros((n, 12), dtype=np.uint64)
    oracle().or_srs(vp(pts), n, vp(tau))
    return pts


def _oracle_commit(pts, sc):
    exp = np.zeros(12, dtype=np.uint64)
    oracle().or_commit(vp(np.ascontiguousarray(pts)), vp(np.ascontiguousarray(sc)), len(sc), vp(exp))
    return exp


@pytest.mark.parametrize("n", [1, 2, 3, 17])
def test_msm_small_n_matrix(ctx, n):
    rng = np.random.default_rng(1000 + n)
    pts = _srs_host(4 * n + 7, n)
    sc = rand_fr_mont_arr(rng, n)
    if n > 2:
        sc[1] = 0
    exp = _oracle_commit(pts[:n], sc)
    assert (_commit_dev(ctx, pts[:n].copy(), sc) == exp).all(), "pnp_commit (per-window layout)"
    assert (_commit_ck(ctx, pts[:n].copy(), sc) == exp).all(), "pnp_commit_ck (folded layout)"
    # the segmented batch: B = 1, then B = 4 sub-ranges of one base set
    dp = to_dev(pts)
    for offs in ([3], [0, n, 2 * n + 1, 3 * n + 7]):
        scs = [rand_fr_mont_arr(rng, n) for _ in offs]
        ds = [to_dev(s) for s in scs]
        got = ctx.commit_segments(dp.data_ptr(), len(pts), offs, [d.data_ptr() for d in ds], n)
        for b, o in enumerate(offs):
            e = _oracle_commit(pts[o:o + n], scs[b])
            assert (np.array(list(got[b].x) + list(got[b].y), dtype=np.uint64) == e).all(), (offs, b)


@pytest.mark.parametrize("n", [2, 4, 16])
def test_commit_evals_small_n(ctx, n):
    from pnp import abi
    rng = np.random.default_rng(77 + n)
    lg = n.bit_length() - 1
    pts = _srs_host(n + 1, 500 + n)
    dp = to_dev(pts)
    ctx.load_commit_key(abi.CommitKeyC(powers_of_g=abi.ptr(dp.data_ptr()), powers_of_gamma_g=abi.ptr(dp.data_ptr())),
                        n + 1, device_ptrs=True)
    ev = rand_fr_mont_arr(rng, n)
    ev[n // 2] = 0
    coeffs = ev.copy()
    oracle().or_ntt(vp(coeffs), lg, 1, 0)
    exp = _oracle_commit(pts[:n], coeffs)
    c = ctx.commit_evals(to_dev(ev).data_ptr(), n)
    assert (np.array(list(c.x) + list(c.y), dtype=np.uint64) == exp).all()


def test_commit_segments_refuses_out_of_range(ctx):
    import pnp
    pts = _srs_host(10, 3)
    dp = to_dev(pts)
    ds = to_dev(rand_fr_mont_arr(np.random.default_rng(3), 4))
    with pytest.raises(pnp.PnpError, match="PNP_E_ARG"):
        ctx.commit_segments(dp.data_ptr(), 10, [7], [ds.data_ptr()], 4)


def test_commit_segments_empty_and_sparse_msms(ctx):
    """A batch whose MSMs leave long runs of empty buckets: one all-zero MSM
    (every bucket of its range empty: an accumulation lane crossing it skips
    2^c buckets at once, msm.hip next_bucket), one with three non-zero scalars
    and one whose scalars are all equal (one bucket per window holds every
    entry), beside a random one — each against the oracle."""
    n = 1 << 14
    rng = np.random.default_rng(4242)
    pts = _srs_host(n, 42)
    dp = to_dev(pts)
    scs = [rand_fr_mont_arr(rng, n), np.zeros((n, 4), dtype=np.uint64), np.zeros((n, 4), dtype=np.uint64),
           np.repeat(rand_fr_mont_arr(rng, 1), n, axis=0)]
    scs[2][[5, 4000, n - 1]] = rand_fr_mont_arr(rng, 3)
    ds = [to_dev(s) for s in scs]
    got = ctx.commit_segments(dp.data_ptr(), n, [0] * 4, [d.data_ptr() for d in ds], n)
    for b in range(4):
        e = _oracle_commit(pts, scs[b])
        assert (np.array(list(got[b].x) + list(got[b].y), dtype=np.uint64) == e).all(), b
