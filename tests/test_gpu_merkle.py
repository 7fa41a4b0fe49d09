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


@pytest.mark.parametrize("height", [4, 8])
def test_synth_merkle_matches_builder(pc, height):
    """pnp_synth_merkle (bench's HEIGHT=15 generator) == tests/merkle_circuit.py
    row for row: wires of every gate, the 9 selectors and 4 sigmas on the whole
    domain, the root."""
    import numpy as np
    import pnp
    from pnp_testlib import fr_mont, ints_to_arr
    from gpu_util import to_dev, empty_dev, from_dev
    import merkle_circuit as mcm
    cp, nodes = mc.merkle_circuit(height, seed=height, pc=pc)
    inp = cp.build()
    n, ng = inp.n, len(cp.rows)
    ctx = pnp.Context(0)
    try:
        leaves = to_dev(ints_to_arr([fr_mont(v) for v in cp.leaves]))
        blind = to_dev(ints_to_arr([fr_mont(v) for v in cp.blind]))
        dnodes = empty_dev(len(nodes))
        w = [empty_dev(ng) for _ in range(4)]
        sel = [empty_dev(n) for _ in range(9)]
        sig = [empty_dev(n) for _ in range(4)]
        root = ctx.synth_merkle(height, mcm.flat_constants(pc), leaves.data_ptr(), blind.data_ptr(),
                                dnodes.data_ptr(), [t.data_ptr() for t in w], [t.data_ptr() for t in sel],
                                [t.data_ptr() for t in sig], n)
        ctx.sync()
        assert root == nodes[0]
        for j, name in enumerate(("w_l", "w_r", "w_o", "w_4")):
            assert np.array_equal(from_dev(w[j]), inp.arrays[name]), name
        exp_nodes = ints_to_arr([fr_mont(v) for v in nodes])
        assert np.array_equal(from_dev(dnodes), exp_nodes)
        names = ("q_l", "q_r", "q_o", "q_4", "q_c", "q_hl", "q_hr", "q_h4", "q_arith")
        for j, name in enumerate(names):
            exp = ints_to_arr([fr_mont(r[0].get(name, 0) % mc.R_MOD) for r in cp.rows] + [0] * (n - ng))
            assert np.array_equal(from_dev(sel[j]), exp), name
        for j, name in enumerate(("left_sigma", "right_sigma", "out_sigma", "fourth_sigma")):
            assert np.array_equal(from_dev(sig[j]), inp.sigma_evals[j]), name
    finally:
        ctx.close()


def _prove_v2_counters(inp, names, env=None):
    import pnp
    ctx = pnp.Context(0)
    try:
        ctx.load_prover_key(inp.pk, inp.n, device_ptrs=False)
        ctx.load_commit_key(inp.ck, inp.n, device_ptrs=False)
        # the first proof goes without the optional tables and builds them in
        # the background (context.h); the second, after it, uses them
        first = ctx.prove_ex(inp.circuit, False, pis_of(inp))
        ctx.sync()
        ctx.kernel_timing(True)
        got = ctx.prove_ex(inp.circuit, False, pis_of(inp))
        assert abi.proof_to_bytes(got) == abi.proof_to_bytes(first)
        return got, {k: ctx.kernel_bytes(k) for k in names}
    finally:
        ctx.close()


def test_merkle_wire_groups_used(pc):
    """Round 1 commits wires a, b, d over the copy-constraint groups of the
    Merkle circuit (csrc/wires.hip: each Poseidon state value sits in three
    consecutive rows of those wires) and round 3 commits z over its runs (z
    is constant over the rows sigma fixes): both grouped paths run and the
    proof is the oracle's byte for byte."""
    cp, _ = mc.merkle_circuit(6, seed=5, pc=pc)
    inp = cp.build()
    exp = inp.oracle_proof()
    got, c = _prove_v2_counters(inp, ["wire_groups_used", "wire_group_fallback", "z_groups_used",
                                      "z_group_fallback"])
    assert abi.proof_to_bytes(got) == abi.proof_to_bytes(exp)
    # z too: constant over the padding rows (sigma fixes them), one scalar per run
    assert c == {"wire_groups_used": 1, "wire_group_fallback": 0, "z_groups_used": 1, "z_group_fallback": 0}


def test_merkle_broken_copy_constraint_falls_back(pc):
    """A witness that breaks a copy constraint (one row of a 3-row Poseidon
    state group changed in wire a): the grouped commitment would differ, so
    the per-proof check sends round 1 back to the row-by-row commitment — the
    proof still equals the oracle's (which commits every row)."""
    cp, _ = mc.merkle_circuit(6, seed=5, pc=pc)
    inp = cp.build()
    va = [r[1][0] for r in cp.rows]
    row = next(i for i in range(1, len(va) - 1) if va[i] == va[i - 1] == va[i + 1] and cp.vals[va[i]])
    w = inp.arrays["w_l"]
    w[row, 0] ^= 1  # still < r: a different field element, in place (the structs point here)
    exp = inp.oracle_proof()
    got, c = _prove_v2_counters(inp, ["wire_groups_used", "wire_group_fallback"])
    assert abi.proof_to_bytes(got) == abi.proof_to_bytes(exp)
    assert c == {"wire_groups_used": 0, "wire_group_fallback": 1}


def test_merkle_wire_groups_off_same_proof(pc, monkeypatch):
    """PNP_WIRE_GROUPS=0 (row-by-row commitments from the evaluations) gives
    the same bytes — checked in a child process, the switch is read once."""
    import subprocess
    import sys
    import os
    code = ("import sys; sys.path[:0] = sys.argv[1:3];"
            "import merkle_circuit as mc, test_gpu_merkle as t; from pnp import abi;"
            "cp, _ = mc.merkle_circuit(5, seed=6); inp = cp.build();"
            "got, c = t._prove_v2_counters(inp, ['wire_groups_used']);"
            "assert c['wire_groups_used'] == 0, c;"
            "assert abi.proof_to_bytes(got) == abi.proof_to_bytes(inp.oracle_proof()); print('ok')")
    here = os.path.dirname(os.path.abspath(__file__))
    pkg = os.path.join(os.path.dirname(here), "zprize23-gpu-submission_amd")
    r = subprocess.run([sys.executable, "-c", code, here, pkg], env=dict(os.environ, PNP_WIRE_GROUPS="0"),
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
