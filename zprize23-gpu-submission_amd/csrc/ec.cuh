// ec.cuh — BLS12-381 G1 (y^2 = x^3 + 4) in XYZZ coordinates, host + device.
//
// The reference accumulates MSM buckets in XYZZ (utils/zkp/cuda/ec/xyzz_t.hpp,
// mixed add 8M+2S :457-460) and folds on the CPU in Jacobian
// (utils/zkp/cpu/collect.h).  Here every stage stays XYZZ:
//   (X, Y, ZZ, ZZZ) ~ affine (X/ZZ, Y/ZZZ), ZZ^3 = ZZZ^2, infinity <=> ZZ = 0.
// Formulas: madd-2008-s, add-2008-s, dbl-2008-s-1, mdbl-2008-s-1 with a = 0,
// with the equal / opposite operand cases handled explicitly so the result is
// correct for any input (repeated bases, P + (-P), infinity).
#pragma once
#include "field.cuh"

// Point operations are out-of-line on the device: each one is ~10-18 Fq
// products (~10-16k instructions); inlining them into unrolled callers made
// compile times explode without a measurable speed benefit.
#define PNP_EC static __host__ __device__ __noinline__

namespace pnp {

struct Xyzz {
    Fq x, y, zz, zzz;
    PNP_HD static Xyzz inf() {
        Xyzz r;
        r.x = Fq::one();
        r.y = Fq::one();
        r.zz = Fq::zero();
        r.zzz = Fq::zero();
        return r;
    }
    PNP_HD bool is_inf() const { return zz.is_zero(); }
};

// 2 * (x, y) affine (mdbl-2008-s-1)
PNP_EC Xyzz dbl_affine(const Fq &x, const Fq &y) {
    Fq u = dbl(y);
    Fq v = sqr(u);
    Fq w = u * v;
    Fq s = x * v;
    Fq x2 = sqr(x);
    Fq m = dbl(x2) + x2;
    Xyzz r;
    r.x = sqr(m) - dbl(s);
    r.y = m * (s - r.x) - w * y;
    r.zz = v;
    r.zzz = w;
    return r;
}

// 2 * P (dbl-2008-s-1)
PNP_EC Xyzz dbl(const Xyzz &p) {
    if (p.is_inf()) return p;
    Fq u = dbl(p.y);
    Fq v = sqr(u);
    Fq w = u * v;
    Fq s = p.x * v;
    Fq x2 = sqr(p.x);
    Fq m = dbl(x2) + x2;
    Xyzz r;
    r.x = sqr(m) - dbl(s);
    r.y = m * (s - r.x) - w * p.y;
    r.zz = v * p.zz;
    r.zzz = w * p.zzz;
    return r;
}

// P + (x2, y2) affine (madd-2008-s)
PNP_EC Xyzz madd(const Xyzz &p, const Fq &x2, const Fq &y2) {
    if (p.is_inf()) {
        Xyzz r;
        r.x = x2;
        r.y = y2;
        r.zz = Fq::one();
        r.zzz = Fq::one();
        return r;
    }
    Fq u2 = x2 * p.zz;
    Fq s2 = y2 * p.zzz;
    Fq P = u2 - p.x;
    Fq R = s2 - p.y;
    if (P.is_zero()) {
        if (R.is_zero()) return dbl_affine(x2, y2);
        return Xyzz::inf();
    }
    Fq pp = sqr(P);
    Fq ppp = P * pp;
    Fq q = p.x * pp;
    Xyzz r;
    r.x = sqr(R) - ppp - dbl(q);
    r.y = R * (q - r.x) - p.y * ppp;
    r.zz = p.zz * pp;
    r.zzz = p.zzz * ppp;
    return r;
}

// P + Q (add-2008-s)
PNP_EC Xyzz add(const Xyzz &p, const Xyzz &q) {
    if (p.is_inf()) return q;
    if (q.is_inf()) return p;
    Fq u1 = p.x * q.zz;
    Fq u2 = q.x * p.zz;
    Fq s1 = p.y * q.zzz;
    Fq s2 = q.y * p.zzz;
    Fq P = u2 - u1;
    Fq R = s2 - s1;
    if (P.is_zero()) {
        if (R.is_zero()) return dbl(p);
        return Xyzz::inf();
    }
    Fq pp = sqr(P);
    Fq ppp = P * pp;
    Fq qq = u1 * pp;
    Xyzz r;
    r.x = sqr(R) - ppp - dbl(qq);
    r.y = R * (qq - r.x) - s1 * ppp;
    r.zz = p.zz * q.zz * pp;
    r.zzz = p.zzz * q.zzz * ppp;
    return r;
}

// host: XYZZ -> affine (x, y) Montgomery; infinity -> (0, one) as the
// reference's to_affine (PLONK/src/point.cu:29-36)
inline void xyzz_to_affine(const Xyzz &p, Fq &x, Fq &y) {
    if (p.is_inf()) {
        x = Fq::zero();
        y = Fq::one();
        return;
    }
    Fq izz = inverse(p.zz);
    Fq izzz = inverse(p.zzz);
    x = p.x * izz;
    y = p.y * izzz;
}

__device__ __forceinline__ void store_xyzz(uint64_t *base, const Xyzz &p) {
    store_fq(base, p.x);
    store_fq(base + 6, p.y);
    store_fq(base + 12, p.zz);
    store_fq(base + 18, p.zzz);
}
__device__ __forceinline__ Xyzz load_xyzz(const uint64_t *base) {
    Xyzz p;
    p.x = load_fq(base);
    p.y = load_fq(base + 6);
    p.zz = load_fq(base + 12);
    p.zzz = load_fq(base + 18);
    return p;
}

}  // namespace pnp
