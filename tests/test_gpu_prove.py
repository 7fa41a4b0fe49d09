"""End-to-end parity: gen_proof on the MI355X vs the CPU restatement, byte for
byte on the 2656-byte ProofC, through both the v1 symbol (host inputs, exactly
as the Rust FFI calls it) and the v2 resident-key API."""
import pytest

from pnp_testlib import Inputs
from pnp import abi

pytestmark = pytest.mark.gpu


def _diff(a, b):
    bad = []
    for name in abi.PROOF_COMMITMENTS:
        ca, cb = getattr(a, name), getattr(b, name)
        if list(ca.x) != list(cb.x) or list(ca.y) != list(cb.y):
            bad.append(name)
    ea, eb = a.evaluations, b.evaluations
    for grp in ("wire_evals", "perm_evals", "lookup_evals", "custom_evals"):
        ga, gb = getattr(ea, grp), getattr(eb, grp)
        for f, _ in ga._fields_:
            if list(getattr(ga, f)) != list(getattr(gb, f)):
                bad.append(f"{grp}.{f}")
    return bad


@pytest.mark.parametrize("lg,seed", [(5, 1), (8, 2), (11, 3)])
def test_gen_proof_v1_parity(lg, seed):
    import pnp
    inp = Inputs(lg, seed)
    exp = inp.oracle_proof()
    lib = pnp.load()
    got = lib.gen_proof(inp.circuit, inp.pk, inp.ck)
    assert _diff(got, exp) == []
    assert abi.proof_to_bytes(got) == abi.proof_to_bytes(exp)


def test_gen_proof_v2_resident(tmp_path):
    import pnp
    inp = Inputs(10, 9, n_gates=1000, pi_pos=17)
    exp = inp.oracle_proof()
    ctx = pnp.Context(0)
    ctx.load_prover_key(inp.pk, inp.n, device_ptrs=False)
    ctx.load_commit_key(inp.ck, inp.n, device_ptrs=False)
    for _ in range(2):  # resident keys are reused across proofs
        got = ctx.prove(inp.circuit, device_ptrs=False)
        assert abi.proof_to_bytes(got) == abi.proof_to_bytes(exp)
    names = [n for n, _ in ctx.stage_times()]
    assert "r4_quotient" in names
    ctx.close()
