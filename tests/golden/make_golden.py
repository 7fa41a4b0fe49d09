"""Generate the committed golden fixtures (tests/golden/*.npz, *.json).

Run in the build container, where /root/reference exists:
    make -C oracle ref && python tests/golden/make_golden.py

Sources of truth (all compiled from the reference's OWN sources by
oracle/ref.mk into oracle/_ref/, never copied):
  * blst (plonk-core/lib/blst/src/server.c + assembly.S; the reference's CPU
    big-integer provider, build.rs:38-54): Fr/Fq Montgomery mul/inverse/
    conversions, G1 scalar multiplication, affine conversion, Pippenger MSM.
  * STROBE-128 / Keccak-f[1600] (plonk-core/lib/PLONK/src/transcript/
    strobe.cpp) driven with the Merlin framing of transcript.cuh:21-64.
  * NTT vectors: the DFT *definition* evaluated with Python big integers over
    the reference's root of unity (PLONK/src/bls12_381/fr.cuh:42) and coset
    generator 7 (fr.cuh:50) — the arkworks/ntt.cuh semantics, independent of
    any FFT code.
Only data (inputs and expected outputs) is written; no reference source.
"""
import ctypes as C
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from pnp_testlib import (R_MOD, Q_MOD, R_FR, R_FQ, REPO, fr_mont, fr_unmont, fr_root,  # noqa: E402
                         to_limbs, from_limbs, ints_to_arr)

REF = os.path.join(REPO, "oracle", "_ref")


def load_refs():
    blst = C.CDLL(os.path.join(REF, "libblst_ref.so"))
    strobe = C.CDLL(os.path.join(REF, "libstrobe_ref.so"))
    blst.blst_p1_affine_generator.restype = C.c_void_p
    blst.blst_p1_generator.restype = C.c_void_p
    blst.blst_p1s_mult_pippenger_scratch_sizeof.restype = C.c_size_t
    blst.blst_p1s_mult_pippenger_scratch_sizeof.argtypes = [C.c_size_t]
    strobe.refm_new.restype = C.c_void_p
    strobe.refm_new.argtypes = [C.c_char_p]
    strobe.refm_free.argtypes = [C.c_void_p]
    strobe.refm_append.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.c_size_t]
    strobe.refm_challenge.argtypes = [C.c_void_p, C.c_char_p, C.c_void_p, C.c_size_t]
    return blst, strobe


def buf(words):
    return (C.c_uint64 * words)()


def arr(b):
    return np.array(list(b), dtype=np.uint64)


def main():
    blst, strobe = load_refs()
    rng = np.random.default_rng(20231015)
    out = {}

    def rnd(mod):
        return int.from_bytes(rng.bytes(64), "little") % mod

    # ---- Fr ----
    N = 64
    fa = [fr_mont(rnd(R_MOD)) for _ in range(N)]
    fb = [fr_mont(rnd(R_MOD)) for _ in range(N)]
    fa[0], fb[1] = 0, fr_mont(1)
    mul, inv, frm = [], [], []
    for a, b in zip(fa, fb):
        ra, rb, rr = buf(4), buf(4), buf(4)
        ra[:] = to_limbs(a, 4)
        rb[:] = to_limbs(b, 4)
        blst.blst_fr_mul(rr, ra, rb)
        mul.append(from_limbs(rr))
        blst.blst_fr_inverse(rr, ra)
        inv.append(from_limbs(rr))
        blst.blst_fr_from(rr, ra)
        frm.append(from_limbs(rr))
    out["fr_a"], out["fr_b"] = ints_to_arr(fa), ints_to_arr(fb)
    out["fr_mul"], out["fr_inv"], out["fr_from"] = ints_to_arr(mul), ints_to_arr(inv), ints_to_arr(frm)

    # ---- Fq ----
    qa = [rnd(Q_MOD) * R_FQ % Q_MOD for _ in range(N)]
    qb = [rnd(Q_MOD) * R_FQ % Q_MOD for _ in range(N)]
    mul, inv = [], []
    for a, b in zip(qa, qb):
        ra, rb, rr = buf(6), buf(6), buf(6)
        ra[:] = to_limbs(a, 6)
        rb[:] = to_limbs(b, 6)
        blst.blst_fp_mul(rr, ra, rb)
        mul.append(from_limbs(rr))
        blst.blst_fp_inverse(rr, ra)
        inv.append(from_limbs(rr))
    out["fq_a"], out["fq_b"] = ints_to_arr(qa, 6), ints_to_arr(qb, 6)
    out["fq_mul"], out["fq_inv"] = ints_to_arr(mul, 6), ints_to_arr(inv, 6)

    # ---- G1 ----
    gen_aff = (C.c_uint64 * 12).from_address(blst.blst_p1_affine_generator())
    out["g1_gen"] = arr(gen_aff)
    gen_j = blst.blst_p1_generator()

    def mult_aff(k):
        pj = buf(18)
        kb = k.to_bytes(32, "little")
        blst.blst_p1_mult(pj, C.c_void_p(gen_j), kb, C.c_size_t(255))
        pa = buf(12)
        blst.blst_p1_to_affine(pa, pj)
        return list(pa), pj

    ks = [rnd(R_MOD) for _ in range(16)]
    ks[0] = 1
    kg = [mult_aff(k)[0] for k in ks]
    out["g1_k"] = ints_to_arr(ks)
    out["g1_kG"] = np.array(kg, dtype=np.uint64)
    # P + Q for pairs of the above (blst_p1_add_or_double, Jacobian)
    sums = []
    for i in range(8):
        _, pj = mult_aff(ks[i])
        _, qj = mult_aff(ks[i + 8])
        s, sa = buf(18), buf(12)
        blst.blst_p1_add_or_double(s, pj, qj)
        blst.blst_p1_to_affine(sa, s)
        sums.append(list(sa))
    out["g1_sum"] = np.array(sums, dtype=np.uint64)

    # ---- MSM (blst_p1s_mult_pippenger) ----
    for n in (1, 2, 3, 17, 64, 257, 1024):
        pts = np.array([mult_aff(rnd(R_MOD))[0] for _ in range(n)], dtype=np.uint64)
        sc = [rnd(R_MOD) for _ in range(n)]
        if n >= 17:
            sc[3] = 0
            sc[5] = R_MOD - 1
            pts[7] = pts[8]  # repeated base
        scal = ints_to_arr(sc)
        scb = b"".join(int(v).to_bytes(32, "little") for v in sc)
        pp = (C.c_void_p * 2)(pts.ctypes.data, None)
        spb = C.create_string_buffer(scb, len(scb))
        sp = (C.c_void_p * 2)(C.addressof(spb), None)
        scratch = C.create_string_buffer(max(1, blst.blst_p1s_mult_pippenger_scratch_sizeof(n)))
        rj, ra = buf(18), buf(12)
        blst.blst_p1s_mult_pippenger(rj, pp, C.c_size_t(n), sp, C.c_size_t(255), scratch)
        blst.blst_p1_to_affine(ra, rj)
        out[f"msm{n}_points"] = pts
        out[f"msm{n}_scalars"] = scal
        out[f"msm{n}_result"] = arr(ra)

    # ---- NTT (DFT definition, python big ints) ----
    for lg in (1, 2, 3, 5, 7):
        n = 1 << lg
        x = [rnd(R_MOD) for _ in range(n)]
        w = fr_root(lg)
        winv = pow(w, -1, R_MOD)
        ninv = pow(n, -1, R_MOD)
        fwd = [sum(x[j] * pow(w, j * k, R_MOD) for j in range(n)) % R_MOD for k in range(n)]
        inv_ = [ninv * sum(x[j] * pow(winv, j * k, R_MOD) for j in range(n)) % R_MOD for k in range(n)]
        cf = [sum(x[j] * pow(7, j, R_MOD) * pow(w, j * k, R_MOD) for j in range(n)) % R_MOD
              for k in range(n)]
        g_inv = pow(7, -1, R_MOD)
        ci = [v * pow(g_inv, k, R_MOD) % R_MOD for k, v in enumerate(inv_)]
        out[f"ntt{lg}_in"] = ints_to_arr([fr_mont(v) for v in x])
        out[f"ntt{lg}_fwd"] = ints_to_arr([fr_mont(v) for v in fwd])
        out[f"ntt{lg}_inv"] = ints_to_arr([fr_mont(v) for v in inv_])
        out[f"ntt{lg}_coset_fwd"] = ints_to_arr([fr_mont(v) for v in cf])
        out[f"ntt{lg}_coset_inv"] = ints_to_arr([fr_mont(v) for v in ci])

    # ---- Keccak-f[1600] ----
    st = rng.integers(0, 2**64, size=25, dtype=np.uint64)
    ks_in = (C.c_uint64 * 25)(*[int(v) for v in st])
    strobe.refm_keccak(ks_in)
    out["keccak_in"] = st
    out["keccak_out"] = arr(ks_in)

    np.savez_compressed(os.path.join(HERE, "golden.npz"), **out)

    # ---- Merlin transcript script (reference Strobe128) ----
    script = [("new", "Merkle tree")]
    msgs = [("pi", 48), ("w_l", 48), ("w_r", 48), ("c", 31), ("zeta", 32), ("long", 400),
            ("c", 31), ("x", 0), ("c", 64), ("t_1", 48), ("c", 31), ("c", 31)]
    h = strobe.refm_new(b"Merkle tree")
    for label, ln in msgs:
        if label == "c":
            o = (C.c_uint8 * ln)()
            lab = f"challenge{len(script)}"
            strobe.refm_challenge(h, lab.encode(), o, ln)
            script.append(("challenge", lab, ln, bytes(o).hex()))
        else:
            m = rng.bytes(ln)
            strobe.refm_append(h, label.encode(), m, len(m))
            script.append(("append", label, m.hex()))
    strobe.refm_free(h)
    with open(os.path.join(HERE, "transcript_script.json"), "w") as f:
        json.dump(script, f, indent=0)
    print("wrote", len(out), "arrays and a", len(script), "step transcript script")


if __name__ == "__main__":
    main()
