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

// Point operations are force-inlined: out-of-line versions pass the 192-byte
// XYZZ result through scratch (512-1184 B/lane of spills, 2 waves/SIMD).
// Callers keep their loops rolled (#pragma unroll 1) so code size and
// compile time stay bounded (each op is ~10-18 Fq products).
#define PNP_EC static __host__ __device__ __forceinline__

namespace pnp {

#ifdef __HIP_DEVICE_COMPILE__
// one definition per translation unit that includes ec.cuh
__device__ __noinline__ Fq fq_mul_ool(Fq a, Fq b) { return a * b; }
#endif

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
    Fq v = fq_mul(u, u);
    Fq w = fq_mul(u, v);
    Fq s = fq_mul(x, v);
    Fq x2 = fq_mul(x, x);
    Fq m = dbl(x2) + x2;
    Xyzz r;
    r.x = fq_mul(m, m) - dbl(s);
    r.y = fq_mul(m, s - r.x) - fq_mul(w, y);
    r.zz = v;
    r.zzz = w;
    return r;
}

// 2 * P (dbl-2008-s-1)
PNP_EC Xyzz dbl(const Xyzz &p) {
    if (p.is_inf()) return p;
    Fq u = dbl(p.y);
    Fq v = fq_mul(u, u);
    Fq w = fq_mul(u, v);
    Fq s = fq_mul(p.x, v);
    Fq x2 = fq_mul(p.x, p.x);
    Fq m = dbl(x2) + x2;
    Xyzz r;
    r.x = fq_mul(m, m) - dbl(s);
    r.y = fq_mul(m, s - r.x) - fq_mul(w, p.y);
    r.zz = fq_mul(v, p.zz);
    r.zzz = fq_mul(w, p.zzz);
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
    Fq u2 = fq_mul(x2, p.zz);
    Fq s2 = fq_mul(y2, p.zzz);
    Fq P = u2 - p.x;
    Fq R = s2 - p.y;
    if (P.is_zero()) {
        if (R.is_zero()) return dbl_affine(x2, y2);
        return Xyzz::inf();
    }
    Fq pp = fq_mul(P, P);
    Fq ppp = fq_mul(P, pp);
    Fq q = fq_mul(p.x, pp);
    Xyzz r;
    r.x = fq_mul(R, R) - ppp - dbl(q);
    r.y = fq_mul(R, q - r.x) - fq_mul(p.y, ppp);
    r.zz = fq_mul(p.zz, pp);
    r.zzz = fq_mul(p.zzz, ppp);
    return r;
}

// P + Q (add-2008-s)
PNP_EC Xyzz add(const Xyzz &p, const Xyzz &q) {
    if (p.is_inf()) return q;
    if (q.is_inf()) return p;
    Fq u1 = fq_mul(p.x, q.zz);
    Fq u2 = fq_mul(q.x, p.zz);
    Fq s1 = fq_mul(p.y, q.zzz);
    Fq s2 = fq_mul(q.y, p.zzz);
    Fq P = u2 - u1;
    Fq R = s2 - s1;
    if (P.is_zero()) {
        if (R.is_zero()) return dbl(p);
        return Xyzz::inf();
    }
    Fq pp = fq_mul(P, P);
    Fq ppp = fq_mul(P, pp);
    Fq qq = fq_mul(u1, pp);
    Xyzz r;
    r.x = fq_mul(R, R) - ppp - dbl(qq);
    r.y = fq_mul(R, qq - r.x) - fq_mul(s1, ppp);
    r.zz = fq_mul(fq_mul(p.zz, q.zz), pp);
    r.zzz = fq_mul(fq_mul(p.zzz, q.zzz), ppp);
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
