"""The lifted parity envelope on the CPU restatement (oracle/prover.c in
prover.rs semantics): proofs of satisfying circuits with every gate family of
the reference prover, general lookups (combine_split) and several public
inputs are ACCEPTED by the restated verifier (oracle/verifier.c, proof.rs:
123-431) — by the SRS trapdoor and, when oracle/_ref is built, by the
reference's own blst pairing — and a witness that breaks one gate is
REJECTED.  The GPU side of the same circuits is tests/test_gpu_general.py."""
import ctypes as C

import numpy as np
import pytest

from circuits import Composer, R_MOD
from pnp_testlib import verify, kzg_points, oracle, fr_unmont, from_limbs, ints_to_arr, vp
from test_verifier import _blst, pairing_ok

FAMILIES = ("arith_qm_pis", "range", "logic", "fbsm", "curve_add", "lookup", "all")


def make_circuit(kind: str, seed: int = 5):
    cp = Composer(seed)
    if kind in ("arith_qm_pis", "all"):
        for k in range(6):
            cp.arith(pi=cp.rnd() if k in (1, 4) else 0)
        # copy constraints: reuse variables of earlier gates
        _, (a, b, c, d) = cp.arith()
        cp.arith(a=c, b=a, d=d)
    if kind in ("range", "all"):
        cp.range_chain(5)
    if kind in ("logic", "all"):
        cp.logic_chain(4, xor=False)
        cp.logic_chain(4, xor=True)
    if kind in ("fbsm", "all"):
        cp.fbsm_chain(6)
    if kind in ("curve_add", "all"):
        cp.curve_add()
        cp.curve_add()
    if kind in ("lookup", "all"):
        cp.lookup_table(11)
        for k in (0, 3, 3, 7, 10, 10, 10):
            cp.lookup(k)
        cp.arith()
    return cp


def pis_of(inp):
    return [(p, v) for p, v in inp.pis]


def check_accepts(inp, proof):
    vk = inp.vk()
    assert verify(vk, proof, pis_of(inp), inp.tau_mont[0])
    blst = _blst()
    if blst is not None:
        rc, pts = kzg_points(vk, proof, pis_of(inp))
        assert rc == 0
        tau = fr_unmont(from_limbs(inp.tau_mont[0]))
        assert pairing_ok(blst, pts[0], pts[1], tau)
        assert pairing_ok(blst, pts[2], pts[3], tau)


@pytest.mark.parametrize("kind", FAMILIES)
def test_general_proof_verifies(kind):
    inp = make_circuit(kind).build()
    proof = inp.oracle_proof()
    # the quotient of a satisfying circuit has degree < 6n... up to the
    # widgets' degree: t_8 stays zero for every family here
    check_accepts(inp, proof)


@pytest.mark.parametrize("kind,row_sel", [("range", "range_selector"), ("logic", "logic_selector"),
                                          ("fbsm", "fixed_group_add_selector"),
                                          ("curve_add", "variable_group_add_selector")])
def test_broken_gate_rejected(kind, row_sel):
    """One wire value of the first gate of the family changed: the quotient is
    no longer a polynomial, the proof must not verify."""
    cp = make_circuit(kind)
    row = next(i for i, r in enumerate(cp.rows) if r[0].get(row_sel))
    va = cp.rows[row][1][0]
    cp.vals[va] = (cp.vals[va] + 1) % R_MOD
    inp = cp.build()
    proof = inp.oracle_proof()
    assert not verify(inp.vk(), proof, pis_of(inp), inp.tau_mont[0])


def test_lookup_query_outside_table_is_an_error():
    cp = make_circuit("lookup")
    r = cp.lookup(0)
    cp.vals[cp.rows[r][1][2]] = 12345  # no such table row
    inp = cp.build()
    lib = oracle()
    out = (C.c_uint8 * 2656)()
    pos, vals = inp.pi_args()
    lib.or_gen_proof_ex.argtypes = [C.c_void_p] * 3 + [C.c_uint64, C.c_void_p, C.c_void_p,
                                                      C.c_char_p, C.c_void_p]
    rc = lib.or_gen_proof_ex(C.byref(inp.circuit), C.byref(inp.pk), C.byref(inp.ck), len(pos),
                             vp(pos), vp(vals), b"Merkle tree", out)
    assert rc == -1  # PNP_E_ARG (Error::ElementNotIndexed in multiset.rs)


def _cs_oracle(t, f):
    n = len(t)
    tt, ff = ints_to_arr(t), ints_to_arr(f)
    h1, h2 = np.zeros((n, 4), np.uint64), np.zeros((n, 4), np.uint64)
    rc = oracle().or_combine_split(vp(tt), vp(ff), C.c_uint64(n), vp(h1), vp(h2))
    return rc, [from_limbs(r) for r in h1], [from_limbs(r) for r in h2]


def test_combine_split_paper_example():
    """multiset.rs:121-124: t {2,4,1,3}, f {2,3,3,2} -> h1 {2,2,1,3}, h2 {2,4,3,3}."""
    rc, h1, h2 = _cs_oracle([2, 4, 1, 3], [2, 3, 3, 2])
    assert rc == 0
    assert h1 == [2, 2, 1, 3] and h2 == [2, 4, 3, 3]


def test_combine_split_repeats_and_first_occurrence_order():
    """Groups follow the FIRST occurrence in t (IndexMap insertion order), odd
    groups alternate h1 / h2 starting with h1."""
    t = [5, 9, 5, 7, 9, 9, 1, 5]
    f = [9, 1, 1, 7, 5, 5, 9, 1]
    rc, h1, h2 = _cs_oracle(t, f)
    assert rc == 0
    # model of multiset.rs:131-180
    from collections import OrderedDict
    cnt = OrderedDict()
    for v in t:
        cnt[v] = cnt.get(v, 0) + 1
    for v in f:
        cnt[v] += 1
    ev, od, par = [], [], 0
    for v, c in cnt.items():
        ev += [v] * (c // 2)
        od += [v] * (c // 2)
        if c % 2:
            (od if par else ev).append(v)
            par ^= 1
    assert h1 == ev and h2 == od
