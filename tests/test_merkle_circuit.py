"""The reference's Poseidon Merkle-tree circuit (tests/merkle_circuit.py, a
restatement of merkle-tree/ + plonk-hashing/) on the CPU restatement: the
constants reproduce the reference's round-number table, the gadget computes
the native hash, the layout has the reference's row count (HEIGHT = 15:
3,161,924 = the headline gate count), and oracle proofs of the real circuit
are accepted by the restated verifier + the reference's blst pairing while a
wrong tree node is rejected.  GPU side: tests/test_gpu_merkle.py."""
import pytest

import merkle_circuit as mc
from test_general import check_accepts, pis_of
from pnp_testlib import verify

# round_numbers.rs:110-135 (t, R_P); R_F = 8 for all
ROUND_NUMBER_KAT = [(2, 55), (3, 55), (4, 56), (5, 56), (6, 56), (7, 56), (8, 57), (9, 57), (10, 57),
                    (11, 57), (12, 57), (13, 57), (14, 57), (15, 57), (16, 59), (17, 59), (25, 59),
                    (37, 60), (65, 61)]


@pytest.fixture(scope="module")
def pc():
    return mc.PoseidonConstants()


def test_round_numbers_match_reference_table():
    for t, rp in ROUND_NUMBER_KAT:
        assert mc.calc_round_numbers(t, True) == (8, rp), t


def test_constants_shape(pc):
    assert (pc.full_rounds, pc.half_full_rounds, pc.partial_rounds) == (8, 4, 55)
    assert len(pc.round_constants) == 3 * (8 + 55)
    assert all(0 <= c < mc.R_MOD for c in pc.round_constants)
    assert len(set(pc.round_constants)) == len(pc.round_constants)
    assert pc.domain_tag == 3
    # Cauchy MDS: symmetric, invertible (mds.rs:59-60)
    M = pc.mds
    assert all(M[i][j] == M[j][i] for i in range(3) for j in range(3))
    det = (M[0][0] * (M[1][1] * M[2][2] - M[1][2] * M[2][1]) - M[0][1] * (M[1][0] * M[2][2] - M[1][2] * M[2][0])
           + M[0][2] * (M[1][0] * M[2][1] - M[1][1] * M[2][0])) % mc.R_MOD
    assert det != 0


def test_gadget_equals_native_hash(pc):
    """zprize_constraints.rs:388-433: the constrained hash equals the native one."""
    cp = mc.MerkleComposer(3)
    for _ in range(3):
        l, r = cp.rnd(), cp.rnd()
        n0 = len(cp.rows)
        out = cp.hash_gadget(pc, cp.var(l), cp.var(r))
        assert len(cp.rows) - n0 == 192
        assert cp.vals[out] == mc.poseidon_hash(pc, l, r)
    assert mc.gate_residuals(cp) == []


@pytest.mark.parametrize("height", [2, 3, 4, 5])
def test_layout_and_satisfied(pc, height):
    cp, nodes = mc.merkle_circuit(height, seed=height, pc=pc)
    assert len(cp.rows) == mc.merkle_rows(height)
    assert mc.gate_residuals(cp) == []
    assert list(cp.pis.items()) == [(len(cp.rows) - 1, (-nodes[0]) % mc.R_MOD)]
    # the selectors the Merkle circuit uses (every other family is zero)
    used = set()
    for q, _ in cp.rows:
        used |= {k for k, v in q.items() if v}
    assert used == {"q_l", "q_r", "q_o", "q_4", "q_c", "q_hl", "q_hr", "q_h4", "q_arith"}


def test_headline_gate_count():
    """HEIGHT = 15 (merkle-tree/src/lib.rs:20) is BASELINE.json's 3,161,924
    gates -> domain 2^22."""
    assert mc.merkle_rows(15) == 3161924
    assert (mc.merkle_rows(15) - 1).bit_length() == 22


def test_merkle_h4_oracle_proof_verifies(pc):
    cp, _ = mc.merkle_circuit(4, seed=11, pc=pc)
    inp = cp.build()
    assert inp.n == 2048 and inp.n_gates == 1356
    proof = inp.oracle_proof()
    check_accepts(inp, proof)


def test_merkle_wrong_node_rejected(pc):
    """A tree node that is not the hash of its children: the witness breaks
    two assert_equal rows and the proof does not verify."""
    cp, _ = mc.merkle_circuit(4, seed=11, pc=pc, corrupt_node=2)
    assert len(mc.gate_residuals(cp)) == 2  # its own row and its parent's
    inp = cp.build()
    proof = inp.oracle_proof()
    assert not verify(inp.vk(), proof, pis_of(inp), inp.tau_mont[0])
