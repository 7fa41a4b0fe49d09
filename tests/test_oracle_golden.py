"""Pin the CPU restatement (oracle/) against the golden fixtures generated from
the reference's own blst / STROBE builds (tests/golden/make_golden.py)."""
import ctypes as C
import json
import os

import numpy as np
import pytest

from pnp_testlib import REPO, oracle, vp

GOLD = np.load(os.path.join(REPO, "tests", "golden", "golden.npz"))


def _bin(fn, a, b, words):
    out = np.zeros((len(a), words), dtype=np.uint64)
    for i in range(len(a)):
        fn(vp(out[i]), vp(np.ascontiguousarray(a[i])), vp(np.ascontiguousarray(b[i])))
    return out


def _un(fn, a, words):
    out = np.zeros((len(a), words), dtype=np.uint64)
    for i in range(len(a)):
        fn(vp(out[i]), vp(np.ascontiguousarray(a[i])))
    return out


def test_fr_mul_inv_from():
    lib = oracle()
    assert (_bin(lib.or_fr_mul, GOLD["fr_a"], GOLD["fr_b"], 4) == GOLD["fr_mul"]).all()
    assert (_un(lib.or_fr_inv, GOLD["fr_a"], 4) == GOLD["fr_inv"]).all()
    assert (_un(lib.or_fr_from_mont, GOLD["fr_a"], 4) == GOLD["fr_from"]).all()


def test_fq_mul_inv():
    lib = oracle()
    assert (_bin(lib.or_fq_mul, GOLD["fq_a"], GOLD["fq_b"], 6) == GOLD["fq_mul"]).all()
    assert (_un(lib.or_fq_inv, GOLD["fq_a"], 6) == GOLD["fq_inv"]).all()


def test_g1_generator_and_mult():
    lib = oracle()
    g = np.zeros(12, dtype=np.uint64)
    lib.or_g1_generator(vp(g))
    assert (g == GOLD["g1_gen"]).all()
    for k, exp in zip(GOLD["g1_k"], GOLD["g1_kG"]):
        out = np.zeros(12, dtype=np.uint64)
        lib.or_g1_mul(vp(out), vp(g), vp(np.ascontiguousarray(k)))
        assert (out == exp).all()


def test_g1_add():
    lib = oracle()
    kg = GOLD["g1_kG"]
    for i in range(8):
        out = np.zeros(12, dtype=np.uint64)
        lib.or_g1_add_affine(vp(out), vp(np.ascontiguousarray(kg[i])), vp(np.ascontiguousarray(kg[i + 8])))
        assert (out == GOLD["g1_sum"][i]).all()


@pytest.mark.parametrize("n", [1, 2, 3, 17, 64, 257, 1024])
def test_msm(n):
    lib = oracle()
    pts = np.ascontiguousarray(GOLD[f"msm{n}_points"])
    sc = np.ascontiguousarray(GOLD[f"msm{n}_scalars"]).copy()
    lib.or_fr_vec_to_mont(vp(sc), n)  # commit() takes Montgomery scalars
    out = np.zeros(12, dtype=np.uint64)
    lib.or_commit(vp(pts), vp(sc), n, vp(out))
    assert (out == GOLD[f"msm{n}_result"]).all()


@pytest.mark.parametrize("lg", [1, 2, 3, 5, 7])
def test_ntt(lg):
    lib = oracle()
    x = GOLD[f"ntt{lg}_in"]
    for inv, coset, key in [(0, 0, "fwd"), (1, 0, "inv"), (0, 1, "coset_fwd"), (1, 1, "coset_inv")]:
        y = x.copy()
        lib.or_ntt(vp(y), lg, inv, coset)
        assert (y == GOLD[f"ntt{lg}_{key}"]).all(), key


def test_keccak():
    lib = oracle()
    st = GOLD["keccak_in"].copy()
    lib.or_keccak_f1600(vp(st))
    assert (st == GOLD["keccak_out"]).all()


def test_transcript_script():
    lib = oracle()
    with open(os.path.join(REPO, "tests", "golden", "transcript_script.json")) as f:
        script = json.load(f)
    t = None
    for step in script:
        if step[0] == "new":
            t = lib.or_transcript_new(step[1].encode())
        elif step[0] == "append":
            m = bytes.fromhex(step[2])
            lib.or_transcript_append_message(t, step[1].encode(), m, len(m))
        else:
            _, label, ln, exp = step
            o = (C.c_uint8 * ln)()
            lib.or_transcript_challenge_bytes(t, label.encode(), o, ln)
            assert bytes(o).hex() == exp, label
    lib.or_transcript_free(t)
