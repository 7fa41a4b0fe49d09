"""Model of the radix-2^29 Fr arithmetic of the NTT passes (csrc/fr29.cuh,
constants tools/gen_fr29.py -> csrc/fr29_consts.inc): every operation mirrors
the device code limb for limb and asserts the bounds the device code relies on
(u32 limbs, u64 column sums, the value bounds of a DIF / DIT pass of up to 8
levels from canonical inputs).  The device kernels themselves are checked
against the oracle by the GPU NTT / LDE / proof tests."""
import os
import random
import re

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
INC = os.path.join(os.path.dirname(HERE), "zprize23-gpu-submission_amd", "csrc", "fr29_consts.inc")
R = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
L, M = 29, (1 << 29) - 1
U32, U64 = 1 << 32, 1 << 64


def _consts():
    txt = open(INC).read()
    c = {m.group(1): [int(x, 16) for x in re.findall(r"0x[0-9a-f]+", m.group(2))]
         for m in re.finditer(r"(R29_\w+)\[9\] = \{([^}]*)\}", txt)}
    kd = re.search(r"R29_KDIF\[8\]\[9\] = \{(.*?)\};", txt, re.S).group(1)
    c["KDIF"] = [[int(x, 16) for x in re.findall(r"0x[0-9a-f]+", row)] for row in re.findall(r"\{([^}]*)\}", kd)]
    c["MU"] = int(re.search(r"R29_MU = (\d+)u", txt).group(1))
    return c


C = _consts()


def val(l):
    return sum(x << (L * i) for i, x in enumerate(l))


def limbs(v):
    return [(v >> (L * i)) & M for i in range(8)] + [v >> (L * 8)]


def norm_ok(l):
    return all(0 <= x <= M for x in l[:8]) and 0 <= l[8] < U32


def from_fr(v):  # 8 x 32-bit words -> 9 limbs (r29_from_fr)
    assert 0 <= v < 2**256
    return limbs(v)


def add(a, b):  # r29_add: normalised sum
    out, c = [], 0
    for i in range(8):
        t = a[i] + b[i] + c
        assert t < U32
        out.append(t & M)
        c = t >> L
    t = a[8] + b[8] + c
    assert t < U32
    return out + [t]


def sub(a, b, K):  # r29_sub: a + K - b, no borrows
    out, c = [], 0
    for i in range(8):
        t = a[i] + K[i] - b[i] + c
        assert 0 <= t < U32
        out.append(t & M)
        c = t >> L
    t = a[8] + K[8] - b[8] + c
    assert 0 <= t < U32
    return out + [t]


def mul(a, b):  # r29_mul: a b 2^-261, product scanning, r_0 = 1, -r^-1 = -1 mod 2^29
    p = C["R29_P"]
    m, out, acc = [0] * 9, [], 0
    for k in range(17):
        for i in range(max(0, k - 8), min(k, 8) + 1):
            acc += a[i] * b[k - i]
            assert acc < U64
        for i in range(max(0, k - 8), min(k, 9)):
            acc += m[i] * p[k - i]
            assert acc < U64
        if k < 9:
            m[k] = (-acc) & M
            acc += m[k]  # m_k * r_0
            assert acc % (1 << L) == 0 and acc < U64
        else:
            out.append(acc & M)
        acc >>= L
    out.append(acc)
    assert acc < U32
    v = val(out)
    assert v == (val(a) * val(b) * pow(2, -261, R)) % R + R * ((v - (val(a) * val(b) * pow(2, -261, R)) % R) // R)
    assert v % R == val(a) * val(b) * pow(2, -261, R) % R
    return out


def canon(x):  # r29_canon: x < 2^264 -> x mod r
    assert norm_ok(x)
    q = (x[8] * C["MU"]) >> 32
    cc = C["R29_C"]
    out, acc = [], 0
    for i in range(8):
        acc += x[i] + q * cc[i]
        assert acc < U64
        out.append(acc & M)
        acc >>= L
    top = acc + x[8] + q * cc[8] - (q << L)
    assert 0 <= acc + x[8] + q * cc[8] < U64 and top >= 0
    y = out + [top]
    assert val(y) == val(x) - q * R and val(y) < 3 * R
    for _ in range(2):  # conditional subtraction of r: z = y + (2^261 - r) >= 2^261 iff y >= r
        z, c = [], 0
        for i in range(8):
            t = y[i] + cc[i] + c
            z.append(t & M)
            c = t >> L
        t = y[8] + cc[8] + c
        ge = t >= (1 << L)
        z.append(t - (1 << L) if ge else t)
        y = z if ge else y
    assert val(y) == val(x) % R
    return y


def test_constants():
    assert val(C["R29_P"]) == R and val(C["R29_C"]) == 2**261 - R
    assert C["MU"] == 2**264 // R
    for lv in range(8):
        assert val(C["KDIF"][lv]) == R << (lv + 1)
    assert val(C["R29_KDIT"]) == 4 * R
    assert val(C["R29_C266"]) == 2**266 % R
    # a 2^256-form table entry -> 2^261 form (ntt.hip k_table_to_r29)
    v = 0x1234567 * 2**256 % R
    assert val(canon(mul(limbs(v), C["R29_C266"]))) == v * 32 % R


def _rand(rng, bound):
    return rng.randrange(bound)


def dif_pass(vals, tw, K=8, pre=None, unit_last=False):
    """One DIF pass of K levels on 2^K canonical inputs (fused pre-twist
    optional); bounds asserted; outputs canonicalised.  unit_last: the last
    level of a whole transform (half size 1, twiddle 1: no product)."""
    x = [from_fr(v) for v in vals]
    if pre is not None:
        x = [mul(a, limbs(p)) for a, p in zip(x, pre)]
    bound = max(val(a) for a in x)
    assert bound < 1.04 * R
    for step in range(K):
        lv = K - 1 - step
        h = 1 << lv
        for blk in range(0, 1 << K, 2 * h):
            for j in range(h):
                a, b = x[blk + j], x[blk + j + h]
                assert val(a) < (1.04 * R) * 2**step and val(b) < (1.04 * R) * 2**step
                s = add(a, b)
                d = sub(a, b, C["KDIF"][step])
                if not (unit_last and step == K - 1):
                    d = mul(d, limbs(tw[(j << (K - 1 - lv)) % len(tw)]))
                x[blk + j], x[blk + j + h] = s, d
    assert all(norm_ok(a) and val(a) < 2**264 for a in x)
    return [val(canon(a)) for a in x]


def dit_pass(vals, tw, K=8, post=None, unit_first=False):
    x = [from_fr(v) for v in vals]
    for step in range(K):
        h = 1 << step
        for blk in range(0, 1 << K, 2 * h):
            for j in range(h):
                a, b = x[blk + j], x[blk + j + h]
                t = b if unit_first and step == 0 else mul(b, limbs(tw[(j << (K - 1 - step)) % len(tw)]))
                assert val(t) < 4 * R
                x[blk + j], x[blk + j + h] = add(a, t), sub(a, t, C["R29_KDIT"])
    if post is not None:
        x = [mul(a, limbs(p)) for a, p in zip(x, post)]
    assert all(norm_ok(a) and val(a) < 2**264 for a in x)
    return [val(canon(a)) for a in x]


def _ref_dft(vals, w, inverse_dit=False):
    n = len(vals)
    return [sum(v * pow(w, i * k, R) for i, v in enumerate(vals)) % R for k in range(n)]


def _brev(i, bits):
    return int(format(i, f"0{bits}b")[::-1], 2)


@pytest.mark.parametrize("worst", [False, True])
def test_dif_pass_matches_dft(worst):
    """A K = 8 DIF pass is the size-256 DFT (bit-reversed out), twiddles in
    2^261 form; worst case: every input r - 1, every twiddle r - 1."""
    K = 8
    rng = random.Random(3)
    g = pow(7, (R - 1) // 256, R)  # a 256th root of unity
    tw = [pow(g, e, R) for e in range(128)]
    tw29 = [t * 2**261 % R for t in tw]
    vals = [R - 1] * 256 if worst else [_rand(rng, R) for _ in range(256)]
    if worst:
        out = dif_pass(vals, [R - 1] * 128, K)  # bounds only
        return
    out = dif_pass(vals, tw29, K)
    ref = _ref_dft(vals, g)
    assert [out[_brev(k, K)] for k in range(256)] == ref


def test_dif_pass_pretwist_bounds():
    rng = random.Random(5)
    vals = [R - 1 - rng.randrange(1000) for _ in range(256)]
    pre = [R - 1 - rng.randrange(1000) for _ in range(256)]
    dif_pass(vals, [R - 1] * 128, 8, pre=pre)


@pytest.mark.parametrize("worst", [False, True])
def test_dit_pass_matches_dft(worst):
    K = 8
    rng = random.Random(4)
    g = pow(7, (R - 1) // 256, R)
    tw = [pow(g, e, R) for e in range(128)]
    tw29 = [t * 2**261 % R for t in tw]
    if worst:
        dit_pass([R - 1] * 256, [R - 1] * 128, K, post=[R - 1] * 256)
        return
    vals = [_rand(rng, R) for _ in range(256)]
    out = dit_pass([vals[_brev(i, K)] for i in range(256)], tw29, K)
    assert out == _ref_dft(vals, g)


def test_canon_edges():
    rng = random.Random(6)
    for v in [0, 1, R - 1, R, R + 1, 2 * R, 3 * R - 1, 2**262, 2**264 - 1, 255 * R, 256 * R - 1] + \
             [rng.randrange(2**264) for _ in range(2000)]:
        assert val(canon(limbs(v))) == v % R


def test_unit_levels_bounds():
    """The half-size-1 level (the last DIF level / first DIT level of a whole
    transform) runs without a product: worst-case bounds still hold."""
    dif_pass([R - 1] * 256, [R - 1] * 128, 8, pre=[R - 1] * 256, unit_last=True)
    dit_pass([R - 1] * 256, [R - 1] * 128, 8, post=[R - 1] * 256, unit_first=True)
    g = pow(7, (R - 1) // 256, R)
    tw29 = [pow(g, e, R) * 2**261 % R for e in range(128)]
    rng = random.Random(9)
    vals = [rng.randrange(R) for _ in range(256)]
    out = dif_pass(vals, tw29, 8, unit_last=True)
    assert [out[_brev(k, 8)] for k in range(256)] == _ref_dft(vals, g)
