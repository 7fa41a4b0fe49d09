"""The reference's own circuit on the MI355X: gen_proof of the Poseidon
Merkle tree (tests/merkle_circuit.py: merkle-tree/ + plonk-hashing/ layout,
HEIGHT = 4 as merkle-tree's configuration (1) and HEIGHT = 8 at 2^15) through
the reference's v1 symbol and the resident v2 API, byte-identical to the CPU
restatement and accepted by the restated verifier + blst pairing
(tests/test_merkle_circuit.py pins the oracle side)."""
import pytest

from pnp import abi
import merkle_circuit as mc
from test_general import check_accepts, pis_of
from test_gpu_prove import _diff

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pc():
    return mc.PoseidonConstants()


def _prove_v2(inp):
    import pnp
    ctx = pnp.Context(0)
    try:
        ctx.load_prover_key(inp.pk, inp.n, device_ptrs=False)
        ctx.load_commit_key(inp.ck, inp.n, device_ptrs=False)
        ctx.kernel_timing(True)
        got = ctx.prove_ex(inp.circuit, False, pis_of(inp))
        fallback = ctx.kernel_bytes("quotient_all_blocks")
        return got, fallback
    finally:
        ctx.close()


def test_merkle_h4_v1_and_v2_equal_oracle(pc):
    import pnp
    cp, _ = mc.merkle_circuit(4, seed=11, pc=pc)
    inp = cp.build()
    assert (inp.n, inp.n_gates) == (2048, 1356)
    exp = inp.oracle_proof()
    v1 = pnp.load().gen_proof(inp.circuit, inp.pk, inp.ck)  # the reference's boundary
    assert _diff(v1, exp) == []
    assert abi.proof_to_bytes(v1) == abi.proof_to_bytes(exp)
    got, fallback = _prove_v2(inp)
    assert abi.proof_to_bytes(got) == abi.proof_to_bytes(exp)
    assert fallback == 0  # deg t < 6n: the 6-block round 4
    check_accepts(inp, got)


def test_merkle_h8_equals_oracle(pc):
    cp, _ = mc.merkle_circuit(8, seed=8, pc=pc)
    inp = cp.build()
    assert (inp.n, inp.n_gates) == (32768, 24516)
    exp = inp.oracle_proof()
    got, fallback = _prove_v2(inp)
    assert _diff(got, exp) == []
    assert fallback == 0
    check_accepts(inp, got)


def test_merkle_wrong_node_all_blocks(pc):
    """An unsatisfied Merkle witness: the round-5 check sends round 4 to all 8
    blocks, the proof is still the reference computation (== oracle) and is
    rejected by the verifier."""
    from pnp_testlib import verify
    cp, _ = mc.merkle_circuit(4, seed=11, pc=pc, corrupt_node=2)
    inp = cp.build()
    exp = inp.oracle_proof()
    got, fallback = _prove_v2(inp)
    assert abi.proof_to_bytes(got) == abi.proof_to_bytes(exp)
    assert fallback == 1
    assert not verify(inp.vk(), got, pis_of(inp), inp.tau_mont[0])
