"""Whole-proof parity pin: proofs of the CPU restatement (oracle/prover.c, byte
-identical to the HIP path by tests/test_gpu_prove.py) are ACCEPTED by a
restatement of the reference verifier (oracle/verifier.c: Proof::verify,
proof.rs:123-431, as driven by merkle-tree/src/main.rs:106-140) and every
single-field corruption is REJECTED.

The KZG pairing check e(L, H) = e(W, [tau]H) is decided twice: with the SRS
trapdoor (L = tau W, exact because e(., H) is injective) and, when the
reference's own blst has been built into oracle/_ref (make -C oracle ref; not
on the GPU box), with blst_miller_loop / blst_final_exp on G2 = the blst
generator and [tau]H = blst_p2_mult."""
import ctypes as C
import os

import numpy as np
import pytest

from pnp import abi
from pnp_testlib import (REPO, Inputs, inputs_pis, inputs_vk, kzg_points, verify, fr_unmont,
                         from_limbs, to_limbs, oracle, vp, R_MOD)

BLST = os.path.join(REPO, "oracle", "_ref", "libblst_ref.so")
FP_ONE_MONT = None


def _blst():
    if not os.path.exists(BLST):
        return None
    lib = C.CDLL(BLST)
    lib.blst_p2_generator.restype = C.c_void_p
    lib.blst_fp12_is_equal.restype = C.c_int
    lib.blst_fp12_is_one.restype = C.c_int
    return lib


def pairing_ok(blst, L, W, tau_canon: int) -> bool:
    """e(L, H) == e(W, [tau] H) with the reference's blst (pairing.c:406-462)."""
    tau_b = (C.c_uint8 * 32)(*tau_canon.to_bytes(32, "little"))
    p2 = (C.c_uint64 * 36)()
    blst.blst_p2_mult(p2, C.c_void_p(blst.blst_p2_generator()), tau_b, 256)
    h_aff = (C.c_uint64 * 24)()
    tau_h = (C.c_uint64 * 24)()
    blst.blst_p2_to_affine(h_aff, C.c_void_p(blst.blst_p2_generator()))
    blst.blst_p2_to_affine(tau_h, p2)

    def gt(P, Q):
        if not any(int(v) for v in P[:6]):  # (0, one) = infinity: e = 1
            return None
        p = (C.c_uint64 * 12)(*[int(v) for v in P])
        ml, fe = (C.c_uint64 * 72)(), (C.c_uint64 * 72)()
        blst.blst_miller_loop(ml, Q, p)
        blst.blst_final_exp(fe, ml)
        return fe

    a, b = gt(L, h_aff), gt(W, tau_h)
    if a is None or b is None:
        return a is None and b is None
    return blst.blst_fp12_is_equal(a, b) == 1


def _tau(inp):
    return fr_unmont(from_limbs(inp.tau_mont[0]))


@pytest.mark.parametrize("lg,seed,gates,pos", [(5, 1, None, 3), (8, 2, None, 3), (11, 3, 2000, 7),
                                               (14, 21, (1 << 14) - 1000, 99)])
def test_oracle_proof_verifies(lg, seed, gates, pos):
    inp = Inputs(lg, seed, n_gates=gates, pi_pos=pos)
    proof = inp.oracle_proof()
    vk = inputs_vk(inp)
    pis = inputs_pis(inp)
    assert verify(vk, proof, pis, inp.tau_mont[0])
    blst = _blst()
    if blst is not None:
        rc, pts = kzg_points(vk, proof, pis)
        assert rc == 0
        tau = _tau(inp)
        assert pairing_ok(blst, pts[0], pts[1], tau)
        assert pairing_ok(blst, pts[2], pts[3], tau)
        # the same pairing rejects a wrong opening
        assert not pairing_ok(blst, pts[0], pts[3], tau)


def _corruptions(proof: abi.ProofC):
    """(name, corrupted copy) for every commitment and every evaluation."""
    lib = oracle()
    raw = abi.proof_to_bytes(proof)
    for name in abi.PROOF_COMMITMENTS:
        p = abi.ProofC.from_buffer_copy(raw)
        c = getattr(p, name)
        aff = np.array(list(c.x) + list(c.y), dtype=np.uint64)
        if not any(int(v) for v in aff[:6]):  # infinity -> the generator
            lib.or_g1_generator(vp(aff))
        else:  # P -> 2P
            two = np.array([2, 0, 0, 0], dtype=np.uint64)
            out = np.zeros(12, dtype=np.uint64)
            lib.or_g1_mul(vp(out), vp(aff), vp(two))
            aff = out
        c.x[:] = [int(v) for v in aff[:6]]
        c.y[:] = [int(v) for v in aff[6:]]
        yield name, p
    ev_off = abi.ProofC.evaluations.offset
    for k in range((len(raw) - ev_off) // 32):
        b = bytearray(raw)
        v = from_limbs(np.frombuffer(bytes(b[ev_off + 32 * k: ev_off + 32 * k + 32]), dtype=np.uint64))
        v = (v + 12345) % R_MOD  # still a reduced residue
        b[ev_off + 32 * k: ev_off + 32 * k + 32] = np.array(to_limbs(v, 4), dtype=np.uint64).tobytes()
        yield f"eval[{k}]", abi.ProofC.from_buffer_copy(bytes(b))


def test_every_corruption_rejected():
    inp = Inputs(6, 5)
    proof = inp.oracle_proof()
    vk = inputs_vk(inp)
    pis = inputs_pis(inp)
    assert verify(vk, proof, pis, inp.tau_mont[0])
    accepted = [name for name, bad in _corruptions(proof) if verify(vk, bad, pis, inp.tau_mont[0])]
    assert accepted == []


def test_wrong_statement_rejected():
    """Wrong public input, wrong PI position, wrong transcript label, and a
    proof of an unsatisfied circuit."""
    inp = Inputs(6, 6)
    proof = inp.oracle_proof()
    vk = inputs_vk(inp)
    (pos, val), = inputs_pis(inp)
    t = inp.tau_mont[0]
    assert verify(vk, proof, [(pos, val)], t)
    assert not verify(vk, proof, [(pos, val + 1)], t)
    assert not verify(vk, proof, [(pos + 1, val)], t)
    assert not verify(vk, proof, [(pos, val)], t, label=b"plonk")
    bad = Inputs(6, 7, satisfying=False)
    assert not verify(inputs_vk(bad), bad.oracle_proof(), inputs_pis(bad), bad.tau_mont[0])


def test_verifier_key_tau_equals_msm_key():
    """or_verifier_key_tau ([p(tau)] G) == or_verifier_key_from_coeffs (MSM over
    the SRS): the trapdoor key bench.py's self-check uses is the real key."""
    from pnp_testlib import verifier_key_tau, VK_POLYS
    inp = Inputs(8, 12, qm_qlookup_evals=True)
    a = inp.arrays
    coeffs = {k: a[k + "_coeffs"] for k in VK_POLYS if k + "_coeffs" in a}
    assert "q_m" in coeffs and "q_lookup" in coeffs
    exp = inputs_vk(inp)
    got = verifier_key_tau(coeffs, inp.n, a["srs"][0], inp.tau_mont[0])
    assert np.array_equal(got, exp)
