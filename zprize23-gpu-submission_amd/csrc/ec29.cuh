// ec29.cuh — G1 XYZZ point arithmetic in radix 2^29 (field29.cuh) for the
// folded MSM's bucket pieces, merge and reduction tree.
//
// Stored points: X, Y < 2^389, ZZ, ZZZ product outputs (< 2^382, limbs
// normalised) or F29_ONE; the point at infinity is all-zero limbs, and any
// ZZ = 0 mod q (0, q or 2q limb for limb: zero29) means infinity.  xadd29 /
// xdbl29 are add-2008-s / dbl-2008-s-1 with the bounds of tests/
// test_field29.py (xadd29, xdbl29 models, asserted at every step).  Equal or
// opposite operands make ZZ3 = ZZ1 ZZ2 (U2 - U1)^2 = 0 mod q, which is detected
// on the (normalised) product output and reported to the caller (xadd29_inf),
// which then recomputes exactly in 32-bit Fq (ec.cuh add handles doubling and
// infinity).
#pragma once
#include "ec.cuh"
#include "field29.cuh"

namespace pnp {

struct Xyzz29 {
    F29 x, y, zz, zzz;
};

__device__ __forceinline__ F29 load29(const uint32_t *p) {
    const uint4 *q = reinterpret_cast<const uint4 *>(p);
    uint4 a = q[0], b = q[1], c = q[2];
    uint2 d = *reinterpret_cast<const uint2 *>(p + 12);
    F29 r;
    r.l[0] = a.x; r.l[1] = a.y; r.l[2] = a.z; r.l[3] = a.w;
    r.l[4] = b.x; r.l[5] = b.y; r.l[6] = b.z; r.l[7] = b.w;
    r.l[8] = c.x; r.l[9] = c.y; r.l[10] = c.z; r.l[11] = c.w;
    r.l[12] = d.x; r.l[13] = d.y;
    return r;
}
__device__ __forceinline__ void store_f29(uint32_t *dst, const F29 &a) {
    uint4 *q = reinterpret_cast<uint4 *>(dst);
    q[0] = make_uint4(a.l[0], a.l[1], a.l[2], a.l[3]);
    q[1] = make_uint4(a.l[4], a.l[5], a.l[6], a.l[7]);
    q[2] = make_uint4(a.l[8], a.l[9], a.l[10], a.l[11]);
    *reinterpret_cast<uint2 *>(dst + 12) = make_uint2(a.l[12], a.l[13]);
}
// a point is 56 u32: x, y, zz, zzz (14 limbs each)
__device__ __forceinline__ Xyzz29 load_xyzz29(const uint32_t *p) {
    Xyzz29 r;
    r.x = load29(p);
    r.y = load29(p + 14);
    r.zz = load29(p + 28);
    r.zzz = load29(p + 42);
    return r;
}
__device__ __forceinline__ void store_xyzz29(uint32_t *p, const Xyzz29 &a) {
    store_f29(p, a.x);
    store_f29(p + 14, a.y);
    store_f29(p + 28, a.zz);
    store_f29(p + 42, a.zzz);
}

// ZZ is a product output (< 2^382 < 3q) or F29_ONE with normalised limbs:
// zero mod q iff it equals 0, q or 2q limb for limb
__device__ __forceinline__ bool zero29(const F29 &v) {
    uint32_t z = 0, a = 0, b = 0;
#pragma unroll
    for (int i = 0; i < 14; i++) {
        z |= v.l[i];
        a |= v.l[i] ^ F29_Q[i];
        b |= v.l[i] ^ F29_Q2[i];
    }
    return z == 0 || a == 0 || b == 0;
}

__device__ __forceinline__ Xyzz29 inf29() {
    Xyzz29 r;
#pragma unroll
    for (int i = 0; i < 14; i++) r.x.l[i] = r.y.l[i] = r.zz.l[i] = r.zzz.l[i] = 0;
    return r;
}

// P + Q (add-2008-s), no exceptional cases: those leave zero29(ZZ3).
// Ordered for short live ranges (the inputs die after the first six
// products): ~130 VGPRs instead of ~250 with both operands kept to the end.
__device__ __forceinline__ Xyzz29 xadd29(const Xyzz29 &p, const Xyzz29 &q) {
    const F29 u1 = mul29(p.x, q.zz);
    const F29 P = sub29(mul29(q.x, p.zz), u1, F29_KB);
    const F29 s1 = mul29(p.y, q.zzz);
    const F29 R = sub29(mul29(q.y, p.zzz), s1, F29_KB);
    const F29 zz12 = mul29(p.zz, q.zz);
    const F29 zzz12 = mul29(p.zzz, q.zzz);
    const F29 pp = sqr29(P);
    const F29 ppp = mul29(P, pp);
    const F29 qq = mul29(u1, pp);
    Xyzz29 r;
    r.zz = mul29(zz12, pp);
    r.zzz = mul29(zzz12, ppp);
    r.x = sub29(sub29(sub29(sqr29(R), ppp, F29_KA), qq, F29_KA), qq, F29_KA);
    // Y3 = R (Q - X3) - S1 PPP as one two-product Montgomery sum
    r.y = mul2_29(R, sub29(qq, r.x, F29_KB), s1, neg29(ppp, F29_KA));
    return r;
}

// 2 P (dbl-2008-s-1, a = 0); P of the prime-order group has Y != 0
__device__ __forceinline__ Xyzz29 xdbl29(const Xyzz29 &p) {
    F29 U;
    {
        uint32_t c = 0;  // Y + Y, carries normalised
#pragma unroll
        for (int i = 0; i < 13; i++) {
            const uint32_t t = p.y.l[i] + p.y.l[i] + c;
            U.l[i] = t & F29_M;
            c = t >> 29;
        }
        U.l[13] = p.y.l[13] + p.y.l[13] + c;
    }
    const F29 V = sqr29(U), W = mul29(U, V), S = mul29(p.x, V), xx = sqr29(p.x);
    F29 M;
    {
        uint32_t c = 0;  // 3 xx
#pragma unroll
        for (int i = 0; i < 13; i++) {
            const uint32_t t = xx.l[i] + xx.l[i] + xx.l[i] + c;
            M.l[i] = t & F29_M;
            c = t >> 29;
        }
        M.l[13] = xx.l[13] + xx.l[13] + xx.l[13] + c;
    }
    Xyzz29 r;
    r.x = sub29(sub29(sqr29(M), S, F29_KA), S, F29_KA);
    r.y = mul2_29(M, sub29(S, r.x, F29_KB), W, neg29(p.y, F29_KB));
    r.zz = mul29(V, p.zz);
    r.zzz = mul29(W, p.zzz);
    return r;
}

__device__ __forceinline__ Xyzz to32(const Xyzz29 &a) {
    Xyzz r;
    r.x = to_fq32(a.x);
    r.y = to_fq32(a.y);
    r.zz = to_fq32(a.zz);
    r.zzz = to_fq32(a.zzz);
    return r;
}
__device__ __forceinline__ Xyzz29 from32(const Xyzz &a) {
    if (a.is_inf()) return inf29();
    Xyzz29 r;
    r.x = from_fq32(a.x);
    r.y = from_fq32(a.y);
    r.zz = from_fq32(a.zz);
    r.zzz = from_fq32(a.zzz);
    return r;
}

// P + Q for inputs that may be infinity; equal / opposite operands (P = 0
// mod q) set *exc and leave a wrong result: the caller then redoes the whole
// reduction in 32-bit Fq (ec.cuh add, exact for every case) — a function
// call here would put the point operands on the stack (1 KB of scratch per
// lane) for a case that random inputs never reach.
__device__ __forceinline__ Xyzz29 xadd29_inf(const Xyzz29 &p, const Xyzz29 &q, uint32_t *exc) {
    if (zero29(p.zz)) return q;
    if (zero29(q.zz)) return p;
    Xyzz29 r = xadd29(p, q);
    if (zero29(r.zz)) *exc = 1u;
    return r;
}
__device__ __forceinline__ Xyzz29 xdbl29_inf(const Xyzz29 &p) {
    if (zero29(p.zz)) return p;
    return xdbl29(p);
}

}  // namespace pnp
