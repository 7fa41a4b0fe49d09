"""The lifted parity envelope on the MI355X: gen_proof of general circuits
(custom gates, lookups with combine_split, several public inputs, a caller
label) through the v2 pnp_prove_ex, byte-identical to the CPU restatement in
prover.rs semantics (tests/test_general.py pins that restatement with the
restated verifier and the reference's blst pairing), and accepted by the
restated verifier; the v1 symbol and pnp_prove agree with pnp_prove_ex on
one public input."""
import ctypes as C

import pytest

from pnp import abi
from test_general import make_circuit, FAMILIES, check_accepts, pis_of
from test_gpu_prove import _diff
from pnp_testlib import Inputs, verify, inputs_vk, inputs_pis

pytestmark = pytest.mark.gpu


def _ctx(inp, device_ptrs=False):
    import pnp
    ctx = pnp.Context(0)
    ctx.load_prover_key(inp.pk, inp.n, device_ptrs=device_ptrs)
    ctx.load_commit_key(inp.ck, inp.n, device_ptrs=device_ptrs)
    return ctx


@pytest.mark.parametrize("kind", FAMILIES)
def test_general_gpu_equals_oracle(kind):
    inp = make_circuit(kind).build()
    exp = inp.oracle_proof()
    ctx = _ctx(inp)
    try:
        ctx.kernel_timing(True)
        got = ctx.prove_ex(inp.circuit, False, pis_of(inp))
        assert _diff(got, exp) == []
        assert abi.proof_to_bytes(got) == abi.proof_to_bytes(exp)
        check_accepts(inp, got)
        # every gate family keeps deg t < 6n: the 6-block round 4 suffices
        assert ctx.kernel_bytes("quotient_all_blocks") == 0
    finally:
        ctx.close()


def test_general_larger_all_gates():
    """2^10 domain with every family repeated (combine_split over long runs of
    the padding value, several odd groups)."""
    from circuits import Composer
    cp = Composer(77)
    cp.lookup_table(100)
    for rep in range(3):
        for k in range(40):
            cp.arith(pi=cp.rnd() if k % 17 == 3 else 0)
        cp.range_chain(20)
        cp.logic_chain(12, xor=rep % 2 == 0)
        cp.fbsm_chain(30)
        cp.curve_add()
        for k in range(60):
            cp.lookup(int(cp.rng.integers(0, 100)))
    inp = cp.build(min_lg=10)
    exp = inp.oracle_proof()
    ctx = _ctx(inp)
    try:
        got = ctx.prove_ex(inp.circuit, False, pis_of(inp))
        assert _diff(got, exp) == []
        check_accepts(inp, got)
    finally:
        ctx.close()


def test_label_and_pi_order():
    """Positions in any order give the BTreeMap order; a different label
    changes the transcript (and the proof), like Transcript::new(label)."""
    inp = make_circuit("arith_qm_pis").build()
    ctx = _ctx(inp)
    try:
        a = ctx.prove_ex(inp.circuit, False, pis_of(inp))
        b = ctx.prove_ex(inp.circuit, False, list(reversed(pis_of(inp))))
        assert abi.proof_to_bytes(a) == abi.proof_to_bytes(b)
        c = ctx.prove_ex(inp.circuit, False, pis_of(inp), label=b"other label")
        assert abi.proof_to_bytes(c) != abi.proof_to_bytes(a)
        exp = inp.oracle_proof(label=b"other label")
        assert abi.proof_to_bytes(c) == abi.proof_to_bytes(exp)
    finally:
        ctx.close()


def test_prove_ex_single_pi_equals_v1():
    import pnp
    inp = Inputs(8, 12)
    ctx = _ctx(inp)
    try:
        a = ctx.prove(inp.circuit, False)
        b = ctx.prove_ex(inp.circuit, False, inputs_pis(inp))
        assert abi.proof_to_bytes(a) == abi.proof_to_bytes(b)
        v1 = pnp.load().gen_proof(inp.circuit, inp.pk, inp.ck)
        assert abi.proof_to_bytes(v1) == abi.proof_to_bytes(a)
        assert verify(inputs_vk(inp), a, inputs_pis(inp), inp.tau_mont[0])
    finally:
        ctx.close()


def test_lookup_query_outside_table_rejected():
    import pnp
    cp = make_circuit("lookup")
    r = cp.lookup(0)
    cp.vals[cp.rows[r][1][2]] = 12345
    inp = cp.build()
    ctx = _ctx(inp)
    try:
        with pytest.raises(pnp.PnpError, match="PNP_E_ARG"):
            ctx.prove_ex(inp.circuit, False, pis_of(inp))
        # the context stays usable
        good = make_circuit("lookup").build()
        ctx.load_prover_key(good.pk, good.n, device_ptrs=False)
        ctx.load_commit_key(good.ck, good.n, device_ptrs=False)
        got = ctx.prove_ex(good.circuit, False, pis_of(good))
        assert abi.proof_to_bytes(got) == abi.proof_to_bytes(good.oracle_proof())
    finally:
        ctx.close()
