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


# ---------------------------------------------------------------- k_quotient29
def mul2(a, b, c, d):  # r29_mul2: (a b + c d) 2^-261, one reduction
    p = C["R29_P"]
    m, out, acc = [0] * 9, [], 0
    for k in range(17):
        for i in range(max(0, k - 8), min(k, 8) + 1):
            acc += a[i] * b[k - i] + c[i] * d[k - i]
            assert acc < U64
        for i in range(max(0, k - 8), min(k, 9)):
            acc += m[i] * p[k - i]
            assert acc < U64
        if k < 9:
            m[k] = (-acc) & M
            acc += m[k]
            assert acc % (1 << L) == 0 and acc < U64
        else:
            out.append(acc & M)
        acc >>= L
    out.append(acc)
    assert acc < U32
    assert val(out) % R == (val(a) * val(b) + val(c) * val(d)) * pow(2, -261, R) % R
    return out


def _mul_in(a, b):  # a product's inputs stay below 2^261 (normalised top limb)
    assert val(a) < 2**261 and val(b) < 2**261 and norm_ok(a) and norm_ok(b)
    return mul(a, b)


def quotient29(x, consts, qm=True, pinv=True):
    """csrc/protocol.hip k_quotient29_ on one point, limb for limb: x = the
    loaded 32-byte values (2^261 form, except vh_inv / l1v / pinv in the
    2^256 form), consts = the 2^261-form constants.  Returns the stored
    (canonical, 2^256-form) value."""
    ld = {k: from_fr(v) for k, v in x.items()}
    cst = {k: limbs(v) for k, v in consts.items()}
    a, b, c, d = ld["a"], ld["b"], ld["c"], ld["d"]

    def pow5(v):
        v2 = _mul_in(v, v)
        return _mul_in(_mul_in(v2, v2), v)

    acc = mul2(a, ld["q_l"], b, ld["q_r"])
    if qm:
        acc = add(acc, _mul_in(_mul_in(a, b), ld["q_m"]))
    acc = add(acc, mul2(c, ld["q_o"], d, ld["q_4"]))
    acc = add(acc, mul2(pow5(a), ld["q_hl"], pow5(b), ld["q_hr"]))
    acc = add(acc, _mul_in(pow5(d), ld["q_h4"]))
    acc = add(acc, ld["q_c"])
    num = _mul_in(acc, ld["q_arith"])
    beta, gamma = cst["beta"], cst["gamma"]
    xb = _mul_in(ld["lin"], beta)
    x2 = add(xb, xb)
    x4 = add(x2, x2)
    x8 = add(x4, x4)
    xb7 = sub(x8, xb, C["KDIF"][0])
    xb13 = add(add(x8, x4), xb)
    xb17 = add(add(x8, x8), xb)
    pa = _mul_in(add(add(xb, a), gamma), add(add(xb7, b), gamma))
    pa = _mul_in(pa, add(add(xb13, c), gamma))
    pa = _mul_in(pa, add(add(xb17, d), gamma))
    f = [add(add(_mul_in(ld[f"sig{j}"], beta), w), gamma) for j, w in enumerate((a, b, c, d))]
    pb = _mul_in(_mul_in(_mul_in(f[0], f[1]), f[2]), f[3])
    zi, zn = ld["zi"], ld["zn"]
    nzn = sub([0] * 9, zn, C["KDIF"][0])
    assert val(pa) < 2**261 and val(pb) < 2**261 and val(nzn) < 2**261
    num = add(num, _mul_in(mul2(pa, zi, pb, nzn), cst["alpha"]))
    l1t = _mul_in(sub(zi, cst["one"], C["KDIF"][0]), cst["alpha2"])
    assert val(num) < 2**261 and val(l1t) < 2**261
    r = mul2(num, ld["vh_inv"], l1t, ld["l1v"])
    if pinv:
        r = add(r, _mul_in(cst["c_pi"], ld["pinv"]))
    assert val(r) < 2**264
    return val(canon(r))


def _quotient_ref(v, k, qm=True, pinv=True):
    """The same numerator in plain field arithmetic (protocol.hip k_quotient_)."""
    a, b, c, d = v["a"], v["b"], v["c"], v["d"]
    gate = (a * v["q_l"] + b * v["q_r"] + (a * b * v["q_m"] if qm else 0) + c * v["q_o"] + d * v["q_4"]
            + pow(a, 5, R) * v["q_hl"] + pow(b, 5, R) * v["q_hr"] + pow(d, 5, R) * v["q_h4"] + v["q_c"])
    num = gate * v["q_arith"]
    x, beta, gamma = v["lin"], k["beta"], k["gamma"]
    pa = (x * beta + a + gamma) * (7 * x * beta + b + gamma) * (13 * x * beta + c + gamma) * \
        (17 * x * beta + d + gamma)
    pb = 1
    for j, w in enumerate((a, b, c, d)):
        pb *= v[f"sig{j}"] * beta + w + gamma
    num += (pa * v["zi"] - pb * v["zn"]) * k["alpha"]
    l1t = (v["zi"] - 1) * k["alpha2"]
    r = num * v["vh_inv"] + l1t * v["l1v"] + (k["c_pi"] * v["pinv"] if pinv else 0)
    return r % R


ARRAYS29 = ("a", "b", "c", "d", "q_l", "q_r", "q_m", "q_o", "q_4", "q_hl", "q_hr", "q_h4", "q_c", "q_arith",
            "lin", "sig0", "sig1", "sig2", "sig3", "zi", "zn")
ARRAYS256 = ("vh_inv", "l1v", "pinv")
CONSTS29 = ("beta", "gamma", "alpha", "alpha2", "one", "c_pi")


@pytest.mark.parametrize("case", ["random", "worst", "qm_off"])
def test_quotient29_model(case):
    """k_quotient29's limb-level model equals the field formula of k_quotient_
    (values in the 2^261 form in, the 2^256 form out), with every column sum
    < 2^64 and every product input < 2^261 asserted; 'worst' takes every
    loaded value and constant r - 1 (the bounds only)."""
    rng = random.Random(11)
    for trial in range(4 if case != "worst" else 1):
        if case == "worst":
            v = {k: R - 1 for k in ARRAYS29 + ARRAYS256}
            kc = {k: R - 1 for k in CONSTS29 if k != "one"}
        else:
            v = {k: rng.randrange(R) for k in ARRAYS29 + ARRAYS256}
            kc = {k: rng.randrange(R) for k in CONSTS29 if k != "one"}
        kc["one"] = 1
        # stored forms: 2^261 for ARRAYS29 and the constants, 2^256 for the final multipliers
        x = {k: v[k] * 2**261 % R for k in ARRAYS29}
        x.update({k: v[k] * 2**256 % R for k in ARRAYS256})
        consts = {k: kc[k] * 2**261 % R for k in CONSTS29}
        if case == "worst":  # the largest stored words everywhere
            x = {k: R - 1 for k in x}
            consts = {k: R - 1 for k in consts}
        qm = case != "qm_off"
        got = quotient29(x, consts, qm=qm)
        if case != "worst":
            assert got == _quotient_ref(v, kc, qm=qm) * 2**256 % R
