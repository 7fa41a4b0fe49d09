"""CPU model of the radix-2^29 Fq arithmetic of csrc/field29.cuh (the MSM
bucket accumulation): the limb-level Montgomery product and lifted-offset
subtraction restated in Python, checked for exactness and for the bounds the
kernel relies on (64-bit column accumulators never overflow, limbs stay
< 2^29, XYZZ coordinates stay below the subtraction offsets) over long chains
of mixed additions, against affine arithmetic on BLS12-381 G1."""
import os
import random
import re

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
INC = os.path.join(HERE, "..", "zprize23-gpu-submission_amd", "csrc", "f29_consts.inc")
Q = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
M29 = (1 << 29) - 1


def _consts():
    txt = open(INC).read()
    arrs = {m.group(1): [int(x.rstrip("u"), 16) for x in m.group(2).split(",")]
            for m in re.finditer(r"(F29_\w+)\[14\] = \{([^}]*)\}", txt)}
    qinv = int(re.search(r"F29_QINV = (0x[0-9a-f]+)u", txt).group(1), 16)
    return arrs, qinv


C, QINV = _consts()


def val(l):
    return sum(x << (29 * i) for i, x in enumerate(l))


def limbs(v):
    return [(v >> (29 * i)) & M29 for i in range(13)] + [v >> (29 * 13)]


def mul29(a, b):
    """mul29 of field29.cuh, limb for limb."""
    assert all(x < 2**29 for x in a + b)
    q = C["F29_Q"]
    m, r, acc = [0] * 14, [0] * 14, 0
    for k in range(27):
        for i in range(max(0, k - 13), min(k, 13) + 1):
            acc += a[i] * b[k - i]
        for i in range(max(0, k - 13), min(k, 14)):
            acc += m[i] * q[k - i]
        if k < 14:
            m[k] = ((acc & 0xFFFFFFFF) * QINV) & M29
            acc += m[k] * q[0]
            assert acc & M29 == 0
        else:
            r[k - 14] = acc & M29
        assert acc < 2**64
        acc >>= 29
    r[13] = acc
    assert acc < 2**29
    return r


def sqr29(a):
    """sqr29 of field29.cuh: cross products against doubled limbs."""
    assert all(x < 2**29 for x in a)
    q = C["F29_Q"]
    a2 = [2 * x for x in a]
    m, r, acc = [0] * 14, [0] * 14, 0
    for k in range(27):
        for i in range(max(0, k - 13), 14):
            if 2 * i < k and k - i <= 13:
                acc += a[i] * a2[k - i]
        if k % 2 == 0:
            acc += a[k // 2] * a[k // 2]
        for i in range(max(0, k - 13), min(k, 14)):
            acc += m[i] * q[k - i]
        if k < 14:
            m[k] = ((acc & 0xFFFFFFFF) * QINV) & M29
            acc += m[k] * q[0]
            assert acc & M29 == 0
        else:
            r[k - 14] = acc & M29
        assert acc < 2**64
        acc >>= 29
    r[13] = acc
    assert acc < 2**29
    return r


def mul2_29(a, b, c, d):
    """mul2_29 of field29.cuh: a b + c d, one reduction."""
    assert all(x < 2**29 for x in a + b + c + d)
    q = C["F29_Q"]
    m, r, acc = [0] * 14, [0] * 14, 0
    for k in range(27):
        for i in range(max(0, k - 13), min(k, 13) + 1):
            acc += a[i] * b[k - i] + c[i] * d[k - i]
        for i in range(max(0, k - 13), min(k, 14)):
            acc += m[i] * q[k - i]
        if k < 14:
            m[k] = ((acc & 0xFFFFFFFF) * QINV) & M29
            acc += m[k] * q[0]
            assert acc & M29 == 0
        else:
            r[k - 14] = acc & M29
        assert acc < 2**64
        acc >>= 29
    r[13] = acc
    assert acc < 2**29
    return r


def sub29(a, b, K):
    r, c = [0] * 14, 0
    for i in range(13):
        t = a[i] + K[i] - b[i] + c
        assert 0 <= t < 2**32
        r[i], c = t & M29, t >> 29
    r[13] = a[13] + K[13] - b[13] + c
    assert r[13] >= 0
    return r


R406 = 1 << 406


def to_m(v):  # integer -> R406 Montgomery limbs
    return limbs(v * R406 % Q)


def from_m(l):
    return val(l) * pow(R406, -1, Q) % Q


def test_constants():
    assert val(C["F29_Q"]) == Q
    assert (QINV * Q) % 2**29 == 2**29 - 1
    assert val(C["F29_ONE"]) == R406 % Q
    assert val(C["F29_C384"]) == 2**384 % Q and val(C["F29_C428"]) == 2**428 % Q
    # zero29 (msm.hip) tests ZZ = 0 mod q against 0, q and 2q limb for limb
    assert val(C["F29_Q2"]) == 2 * Q and all(x <= M29 for x in C["F29_Q2"])
    for k, lo in (("F29_KA", 386), ("F29_KB", 389)):
        v = val(C[k])
        assert v % Q == 0 and 2**lo <= v < 2**(lo + 1)
        assert all(2**29 <= x < 2**30 for x in C[k][:13])


def test_mul_exact_and_bounded():
    rnd = random.Random(1)
    for _ in range(300):
        a, b = rnd.randrange(2**391), rnd.randrange(2**391)
        r = mul29(limbs(a), limbs(b))
        assert val(r) % Q == a * b * pow(R406, -1, Q) % Q
        assert val(r) < 2**382
        s = sqr29(limbs(a))
        assert val(s) == val(mul29(limbs(a), limbs(a)))
        c, d = rnd.randrange(2**391), rnd.randrange(2**391)
        t = mul2_29(limbs(a), limbs(b), limbs(c), limbs(d))
        assert val(t) % Q == (a * b + c * d) * pow(R406, -1, Q) % Q
        assert val(t) < 2**382
    top = limbs(2**391 - 1)  # every limb at its maximum: worst column sums
    assert val(sqr29(top)) == val(mul29(top, top))
    mul2_29(top, top, top, top)


# ---- G1 (y^2 = x^3 + 4) affine reference
G1X = 0x17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb
G1Y = 0x08b3f481e3aaa0f1a09e30ed741d8ae4fcf5e095d5d00af600db18cb2c04b3edd03cc744a2888ae40caa232946c5e7e1


def aff_add(p, q):
    (x1, y1), (x2, y2) = p, q
    lam = (y2 - y1) * pow(x2 - x1, -1, Q) % Q
    x3 = (lam * lam - x1 - x2) % Q
    return x3, (lam * (x1 - x3) - y1) % Q


def madd29(p, x2, y2):
    """madd29 of msm.hip with the bounds of field29.cuh asserted."""
    KA, KB = C["F29_KA"], C["F29_KB"]
    X, Y, ZZ, ZZZ = p
    for v in (X, Y):
        assert val(v) < 2**389
    u2, s2 = mul29(x2, ZZ), mul29(y2, ZZZ)
    P, R = sub29(u2, X, KB), sub29(s2, Y, KB)
    assert val(P) < 2**391 and val(R) < 2**391
    pp = sqr29(P)
    ppp = mul29(P, pp)
    q = mul29(X, pp)
    x3 = sub29(sub29(sub29(sqr29(R), ppp, KA), q, KA), q, KA)
    assert val(x3) < 2**389
    t = sub29(q, x3, KB)
    assert val(t) < 2**391
    y3 = mul2_29(R, t, Y, sub29([0] * 14, ppp, KA))
    assert val(y3) < 2**382
    return x3, y3, mul29(ZZ, pp), mul29(ZZZ, ppp)


@pytest.mark.parametrize("seed", [3, 4])
def test_madd_chain(seed):
    rnd = random.Random(seed)
    pts, P = [], (G1X, G1Y)
    for _ in range(24):  # distinct multiples of G
        k = rnd.randrange(1, 2**64)
        acc = None
        base, e = P, k
        while e:
            if e & 1:
                acc = base if acc is None else aff_add(acc, base)
            x, y = base
            lam = 3 * x * x * pow(2 * y, -1, Q) % Q
            x3 = (lam * lam - 2 * x) % Q
            base = (x3, (lam * (x - x3) - y) % Q)
            e >>= 1
        pts.append(acc)
    ref = pts[0]
    acc = (to_m(pts[0][0]), to_m(pts[0][1]), to_m(1), to_m(1))
    for x, y in pts[1:]:
        neg = rnd.random() < 0.5
        ym = to_m(y)
        if neg:
            ym = sub29([0] * 14, ym, C["F29_KA"])
            y = (-y) % Q
        acc = madd29(acc, to_m(x), ym)
        ref = aff_add(ref, (x, y))
    X, Y, ZZ, ZZZ = (from_m(v) for v in acc)
    assert X * pow(ZZ, -1, Q) % Q == ref[0]
    assert Y * pow(ZZZ, -1, Q) % Q == ref[1]


# ---- general XYZZ addition / doubling in radix 2^29 (ec29.cuh: the bucket
# merge and the reduction tree)
def add29n(a, b):
    """a + b with carries normalised (limbs < 2^29)."""
    r, c = [0] * 14, 0
    for i in range(13):
        t = a[i] + b[i] + c
        r[i], c = t & M29, t >> 29
    r[13] = a[13] + b[13] + c
    return r


def xadd29(p, q):
    """add-2008-s on XYZZ inputs, no exceptional cases (they leave ZZ = 0 mod q)."""
    KA, KB = C["F29_KA"], C["F29_KB"]
    X1, Y1, ZZ1, ZZZ1 = p
    X2, Y2, ZZ2, ZZZ2 = q
    for v in (X1, Y1, X2, Y2):  # stored coordinates (same bounds as madd29)
        assert val(v) < 2**389
    for v in (ZZ1, ZZZ1, ZZ2, ZZZ2):  # product outputs
        assert val(v) < 2**382
    u1, u2 = mul29(X1, ZZ2), mul29(X2, ZZ1)
    s1, s2 = mul29(Y1, ZZZ2), mul29(Y2, ZZZ1)
    P, R = sub29(u2, u1, KB), sub29(s2, s1, KB)
    assert val(P) < 2**391 and val(R) < 2**391  # product inputs
    pp = sqr29(P)
    ppp = mul29(P, pp)
    q_ = mul29(u1, pp)
    x3 = sub29(sub29(sub29(sqr29(R), ppp, KA), q_, KA), q_, KA)
    assert val(x3) < 2**389
    t = sub29(q_, x3, KB)
    assert val(t) < 2**391
    y3 = mul2_29(R, t, s1, sub29([0] * 14, ppp, KA))
    assert val(y3) < 2**382
    return x3, y3, mul29(mul29(ZZ1, ZZ2), pp), mul29(mul29(ZZZ1, ZZZ2), ppp)


def xdbl29(p):
    """dbl-2008-s-1 (a = 0) on an XYZZ input."""
    KA, KB = C["F29_KA"], C["F29_KB"]
    X, Y, ZZ, ZZZ = p
    assert val(X) < 2**389 and val(Y) < 2**389
    assert val(ZZ) < 2**382 and val(ZZZ) < 2**382
    U = add29n(Y, Y)
    assert val(U) < 2**391
    V = sqr29(U)
    W = mul29(U, V)
    S = mul29(X, V)
    xx = sqr29(X)
    M = add29n(add29n(xx, xx), xx)
    assert val(M) < 2**391
    x3 = sub29(sub29(sqr29(M), S, KA), S, KA)
    assert val(x3) < 2**389
    t, ny = sub29(S, x3, KB), sub29([0] * 14, Y, KB)
    assert val(t) < 2**391 and val(ny) < 2**391
    y3 = mul2_29(M, t, W, ny)
    assert val(y3) < 2**382
    return x3, y3, mul29(V, ZZ), mul29(W, ZZZ)


def _aff(p):
    X, Y, ZZ, ZZZ = (from_m(v) for v in p)
    return X * pow(ZZ, -1, Q) % Q, Y * pow(ZZZ, -1, Q) % Q


def _dbl_aff(p):
    x, y = p
    lam = 3 * x * x * pow(2 * y, -1, Q) % Q
    x3 = (lam * lam - 2 * x) % Q
    return x3, (lam * (x - x3) - y) % Q


def _mulg(k):
    acc, base = None, (G1X, G1Y)
    while k:
        if k & 1:
            acc = base if acc is None else aff_add(acc, base)
        base = _dbl_aff(base)
        k >>= 1
    return acc


def test_xadd_xdbl():
    rnd = random.Random(7)
    a, b = _mulg(rnd.randrange(1, 2**64)), _mulg(rnd.randrange(1, 2**64))
    A = (to_m(a[0]), to_m(a[1]), to_m(1), to_m(1))
    B = (to_m(b[0]), to_m(b[1]), to_m(1), to_m(1))
    AB = xadd29(A, B)
    assert _aff(AB) == aff_add(a, b)
    assert _aff(xdbl29(A)) == _dbl_aff(a)
    assert _aff(xadd29(AB, A)) == aff_add(aff_add(a, b), a)
    assert _aff(xdbl29(AB)) == _dbl_aff(aff_add(a, b))


@pytest.mark.parametrize("seed", [11, 12])
def test_xadd_xdbl_chain(seed):
    """Long random mixes of general additions and doublings (the bucket
    reduction's operation mix), every bound asserted at every step."""
    rnd = random.Random(seed)
    pts = [_mulg(rnd.randrange(1, 2**64)) for _ in range(6)]
    X = [(to_m(x), to_m(y), to_m(1), to_m(1)) for x, y in pts]
    ref = list(pts)
    for _ in range(40):
        i, j = rnd.randrange(len(X)), rnd.randrange(len(X))
        if i == j or rnd.random() < 0.3:
            X[i] = xdbl29(X[i])
            ref[i] = _dbl_aff(ref[i])
        else:
            X[i] = xadd29(X[i], X[j])
            ref[i] = aff_add(ref[i], ref[j])
        assert _aff(X[i]) == ref[i]


# ---- the quad-lane forms of the tree's top levels (msm_reduce.hip xadd29w /
# xdbl29w): the same products issued four at a time, squares as mul29, and
# Y3 as two products summed instead of one two-product reduction
def xadd29w(p, q):
    KA, KB = C["F29_KA"], C["F29_KB"]
    X1, Y1, ZZ1, ZZZ1 = p
    X2, Y2, ZZ2, ZZZ2 = q
    for v in (X1, Y1, X2, Y2):
        assert val(v) < 2**389
    for v in (ZZ1, ZZZ1, ZZ2, ZZZ2):
        assert val(v) < 2**382
    u1, u2, s1, s2 = mul29(X1, ZZ2), mul29(X2, ZZ1), mul29(Y1, ZZZ2), mul29(Y2, ZZZ1)
    P, R = sub29(u2, u1, KB), sub29(s2, s1, KB)
    assert val(P) < 2**391 and val(R) < 2**391
    pp, rr, zz12, zzz12 = mul29(P, P), mul29(R, R), mul29(ZZ1, ZZ2), mul29(ZZZ1, ZZZ2)
    ppp, q_, zz3 = mul29(P, pp), mul29(u1, pp), mul29(zz12, pp)
    x3 = sub29(sub29(sub29(rr, ppp, KA), q_, KA), q_, KA)
    assert val(x3) < 2**389
    t, nppp = sub29(q_, x3, KB), sub29([0] * 14, ppp, KA)
    assert val(t) < 2**391 and val(nppp) < 2**391
    y3 = add29n(mul29(R, t), mul29(s1, nppp))
    assert val(y3) < 2**383 and all(x < 2**29 for x in y3[:13])
    return x3, y3, zz3, mul29(zzz12, ppp)


def xdbl29w(p):
    KA, KB = C["F29_KA"], C["F29_KB"]
    X, Y, ZZ, ZZZ = p
    assert val(X) < 2**389 and val(Y) < 2**389
    assert val(ZZ) < 2**382 and val(ZZZ) < 2**382
    U = add29n(Y, Y)
    assert val(U) < 2**391
    V, xx = mul29(U, U), mul29(X, X)
    M = add29n(add29n(xx, xx), xx)
    assert val(M) < 2**391
    W, S, mm, zz3 = mul29(U, V), mul29(X, V), mul29(M, M), mul29(V, ZZ)
    x3 = sub29(sub29(mm, S, KA), S, KA)
    assert val(x3) < 2**389
    t, ny = sub29(S, x3, KB), sub29([0] * 14, Y, KB)
    assert val(t) < 2**391 and val(ny) < 2**391
    y3 = add29n(mul29(M, t), mul29(W, ny))
    assert val(y3) < 2**383
    return x3, y3, zz3, mul29(W, ZZZ)


@pytest.mark.parametrize("seed", [21, 22])
def test_quad_forms_chain(seed):
    """The reduction tree's operation mix through the quad-lane forms, fed
    with the serial forms' outputs and their own (both Y bounds), every bound
    asserted, against affine arithmetic."""
    rnd = random.Random(seed)
    pts = [_mulg(rnd.randrange(1, 2**64)) for _ in range(6)]
    X = [(to_m(x), to_m(y), to_m(1), to_m(1)) for x, y in pts]
    ref = list(pts)
    for step in range(48):
        i, j = rnd.randrange(len(X)), rnd.randrange(len(X))
        wide = step % 3 != 0
        if i == j or rnd.random() < 0.3:
            X[i] = (xdbl29w if wide else xdbl29)(X[i])
            ref[i] = _dbl_aff(ref[i])
        else:
            X[i] = (xadd29w if wide else xadd29)(X[i], X[j])
            ref[i] = aff_add(ref[i], ref[j])
        assert _aff(X[i]) == ref[i]
