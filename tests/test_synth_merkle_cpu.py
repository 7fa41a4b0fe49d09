"""CPU mirror of the bench's Merkle generator (oracle/synth.c or_synth_merkle,
which restates csrc/synth.hip pnp_synth_merkle) against the row-for-row
builder of the reference's circuit (tests/merkle_circuit.py): wires of every
gate, the 9 selectors and 4 sigmas on the whole domain, the tree nodes and
the root.  This is what lets the CPU restatement prove the bench's own
HEIGHT=15 instance (tests/golden/merkle_h15_seed1.json)."""
import ctypes as C

import numpy as np
import pytest

import merkle_circuit as mc
from pnp_testlib import fr_mont, ints_to_arr, vp
from synth_cpu import SyntheticCPU, _lib, merkle_gates


@pytest.fixture(scope="module")
def pc():
    return mc.PoseidonConstants()


@pytest.mark.parametrize("height", [3, 4, 6])
def test_or_synth_merkle_matches_builder(pc, height):
    cp, nodes = mc.merkle_circuit(height, seed=height, pc=pc)
    inp = cp.build()
    n, ng = inp.n, len(cp.rows)
    assert ng == merkle_gates(height)
    lib = _lib()
    leaves = ints_to_arr([fr_mont(v) for v in cp.leaves])
    blind = ints_to_arr([fr_mont(v) for v in cp.blind])
    consts = ints_to_arr([fr_mont(v) for v in mc.flat_constants(pc)])
    dnodes = np.zeros((len(nodes), 4), dtype=np.uint64)
    w = [np.zeros((ng, 4), dtype=np.uint64) for _ in range(4)]
    sel = [np.zeros((n, 4), dtype=np.uint64) for _ in range(9)]
    sig = [np.zeros((n, 4), dtype=np.uint64) for _ in range(4)]
    root = np.zeros(4, dtype=np.uint64)
    rc = lib.or_synth_merkle(height, vp(consts), vp(leaves), vp(blind), vp(dnodes),
                             (C.c_void_p * 4)(*[x.ctypes.data for x in w]),
                             (C.c_void_p * 9)(*[x.ctypes.data for x in sel]),
                             (C.c_void_p * 4)(*[x.ctypes.data for x in sig]), n, vp(root))
    assert rc == 0
    assert sum(int(root[k]) << (64 * k) for k in range(4)) == nodes[0]
    assert np.array_equal(dnodes, ints_to_arr([fr_mont(v) for v in nodes]))
    for j, name in enumerate(("w_l", "w_r", "w_o", "w_4")):
        assert np.array_equal(w[j], inp.arrays[name]), name
    names = ("q_l", "q_r", "q_o", "q_4", "q_c", "q_hl", "q_hr", "q_h4", "q_arith")
    for j, name in enumerate(names):
        exp = ints_to_arr([fr_mont(r[0].get(name, 0) % mc.R_MOD) for r in cp.rows] + [0] * (n - ng))
        assert np.array_equal(sel[j], exp), name
    for j, name in enumerate(("left_sigma", "right_sigma", "out_sigma", "fourth_sigma")):
        assert np.array_equal(sig[j], inp.sigma_evals[j]), name


def test_or_synth_merkle_rejects_small_domain(pc):
    lib = _lib()
    z = np.zeros((1 << 12, 4), dtype=np.uint64)
    ptr4 = (C.c_void_p * 4)(*[z.ctypes.data] * 4)
    ptr9 = (C.c_void_p * 9)(*[z.ctypes.data] * 9)
    assert lib.or_synth_merkle(5, vp(z), vp(z), vp(z), vp(z), ptr4, ptr9, ptr4, 1 << 11, vp(z)) == -1


def test_synthetic_cpu_merkle_proof_verifies():
    """SyntheticCPU(circuit="merkle") at HEIGHT 4 (2^11): the CPU restatement's
    proof of the bench's own instance is accepted by the restated verifier."""
    from pnp_testlib import verify
    syn = SyntheticCPU(11, 0, seed=1, circuit="merkle")
    assert syn.gates == 1356 and syn.pi_pos == 1355
    proof = syn.oracle_proof()
    assert verify(syn.vk(), proof, syn.pis(), syn.tau_mont[0])
    # a different seed is a different instance (leaves, blinding, root)
    other = SyntheticCPU(11, 0, seed=2, circuit="merkle")
    assert other.root != syn.root
