"""Commitments from evaluations against the commit key in the Lagrange basis
(csrc/lagrange.hip, pnp_commit_evals — what gen_proof's round 1 uses for the
wire commitments):

  * equal to the oracle's MSM over the coefficients iNTT(evals) (oracle/g1.c
    or_commit, oracle/ntt.c or_ntt) at 2^1 .. 2^13, with zero runs and zero
    tails like a padded witness, on a key longer than n;
  * equal to the folded monomial-key MSM (pnp_commit_ck, pinned against the
    oracle at 2^22 by test_gpu_full.py) over the GPU iNTT's coefficients at
    the headline size 2^22, with the Merkle circuit's zero tail;
  * a degenerate key (tau = 1, a point of the subgroup: L_i(tau) = 0 for
    i != 0) is refused with PNP_E_ARG rather than producing wrong points, and
    gen_proof then commits from coefficients (the prover's fallback)."""
import time

import numpy as np
import pytest

from gpu_util import empty_dev, from_dev, to_dev
from pnp_testlib import fr_mont, oracle, to_limbs, vp

pytestmark = pytest.mark.gpu


def _ck(addr):
    from pnp import abi
    return abi.CommitKeyC(powers_of_g=abi.ptr(addr), powers_of_gamma_g=abi.ptr(addr))


def _srs(ctx, m, tau_mont):
    srs = empty_dev(m, 12)
    ctx.srs(srs.data_ptr(), m, to_limbs(tau_mont, 4))
    ctx.sync()
    return srs


def _evals(ctx, n, seed):
    d = empty_dev(n)
    ctx.random_fr(d.data_ptr(), n, seed)
    ctx.sync()
    h = from_dev(d).copy()
    h[n - n // 4:] = 0  # padding rows
    h[::5] = 0          # zero-variable slots
    return h


def _pt(c):
    return np.array(list(c.x) + list(c.y), dtype=np.uint64)


@pytest.mark.parametrize("lg", [1, 2, 5, 10, 13])
def test_commit_evals_vs_oracle(lg):
    import pnp
    n = 1 << lg
    ctx = pnp.Context(0)
    try:
        srs = _srs(ctx, n + 3, fr_mont(0x1234567890ABCDEF1357 + lg))
        pts = from_dev(srs, 12).copy()
        ctx.load_commit_key(_ck(srs.data_ptr()), n + 3, device_ptrs=True)
        ev = _evals(ctx, n, 17 + lg)
        coeffs = ev.copy()
        oracle().or_ntt(vp(coeffs), lg, 1, 0)
        exp = np.zeros(12, dtype=np.uint64)
        oracle().or_commit(vp(pts[:n].copy()), vp(coeffs), n, vp(exp))
        d = to_dev(ev)
        assert (_pt(ctx.commit_evals(d.data_ptr(), n)) == exp).all()
        # the basis is kept: a second polynomial over the same key
        ev2 = _evals(ctx, n, 99 + lg)
        c2 = ev2.copy()
        oracle().or_ntt(vp(c2), lg, 1, 0)
        oracle().or_commit(vp(pts[:n].copy()), vp(c2), n, vp(exp))
        d2 = to_dev(ev2)
        assert (_pt(ctx.commit_evals(d2.data_ptr(), n)) == exp).all()
    finally:
        ctx.close()


def test_commit_evals_2e22_vs_monomial_key():
    import pnp
    lg, n = 22, 1 << 22
    ctx = pnp.Context(0)
    try:
        tau = empty_dev(1)
        ctx.random_fr(tau.data_ptr(), 1, 4242)
        ctx.sync()
        srs = empty_dev(n, 12)
        ctx.srs(srs.data_ptr(), n, [int(v) for v in from_dev(tau)[0]])
        ctx.sync()
        ctx.load_commit_key(_ck(srs.data_ptr()), n, device_ptrs=True)
        ev = _evals(ctx, n, 7)
        ev[3161924:] = 0  # the HEIGHT = 15 Merkle circuit's padding rows
        d_ev = to_dev(ev)
        d_c = to_dev(ev)
        ctx.ntt(d_c.data_ptr(), lg, inverse=True)
        ctx.sync()
        t0 = time.time()
        got = _pt(ctx.commit_evals(d_ev.data_ptr(), n))
        t1 = time.time()
        print(f"Lagrange basis of 2^22 points + folded table + first commitment: {t1 - t0:.2f} s")
        exp = _pt(ctx.commit_ck(d_c.data_ptr(), n))
        assert (got == exp).all()
        t2 = time.time()
        assert (_pt(ctx.commit_evals(d_ev.data_ptr(), n)) == exp).all()
        print(f"second commitment from evaluations: {time.time() - t2:.3f} s")
    finally:
        ctx.close()


def test_commit_evals_degenerate_key_refused():
    import pnp
    n = 1 << 6
    ctx = pnp.Context(0)
    try:
        srs = _srs(ctx, n, fr_mont(1))  # tau = 1 = omega^0: every [tau^j] G = G
        ctx.load_commit_key(_ck(srs.data_ptr()), n, device_ptrs=True)
        ev = _evals(ctx, n, 3)
        d = to_dev(ev)
        with pytest.raises(pnp.PnpError, match="PNP_E_ARG"):
            ctx.commit_evals(d.data_ptr(), n)
    finally:
        ctx.close()


def test_prover_coefficient_commitments_same_proof():
    """gen_proof with the Lagrange basis switched off (PNP_LAGRANGE=0: the
    path a degenerate key takes) returns the same bytes as the oracle, like
    the default path does (test_gpu_merkle.py); run in a child process, the
    switch is read once per process."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    code = (
        "import sys; sys.path[:0] = [%r, %r]\n"
        "import merkle_circuit as mc\n"
        "from test_general import pis_of\n"
        "from pnp import abi\n"
        "import pnp\n"
        "cp, _ = mc.merkle_circuit(4, seed=11)\n"
        "inp = cp.build()\n"
        "exp = inp.oracle_proof()\n"
        "ctx = pnp.Context(0)\n"
        "ctx.load_prover_key(inp.pk, inp.n, device_ptrs=False)\n"
        "ctx.load_commit_key(inp.ck, inp.n, device_ptrs=False)\n"
        "got = ctx.prove_ex(inp.circuit, False, pis_of(inp))\n"
        "ctx.close()\n"
        "assert abi.proof_to_bytes(got) == abi.proof_to_bytes(exp)\n"
        "print('SAME')\n"
    ) % (here, os.path.join(os.path.dirname(here), "zprize23-gpu-submission_amd"))
    env = dict(os.environ, PNP_LAGRANGE="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "SAME" in r.stdout
