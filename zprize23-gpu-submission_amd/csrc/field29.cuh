// field29.cuh — BLS12-381 Fq in radix 2^29 (14 limbs), for the MSM bucket
// accumulation on gfx950.
//
// Why: the 32-bit-limb Montgomery product (field.cuh) spends one
// v_addc_co_u32 per v_mad_u64_u32 to carry the 96-bit column sums, and on
// gfx950 both cost ~4.3 cycles per wave64 instruction (tools/ubench_ops.hip).
// With 29-bit limbs every product is < 2^58 and a whole column (<= 28
// products + carry) fits a 64-bit accumulator, so the product is 392 bare
// v_mad_u64_u32 plus a shift/mask per column: ~25% fewer issue cycles.
//
// Representation: value V = sum l_i 2^(29 i), every limb < 2^29, Montgomery
// with R = 2^406, NOT reduced: a product of inputs < 2^391 is < 2^382, and the
// subtractions add a multiple of q (F29_KA ~ 2^386 > any product, F29_KB ~
// 2^389 > any stored coordinate) whose limbs are "lifted" into [2^29, 2^30),
// so no limb ever borrows and no conditional reduction is needed.  The bounds
// are tracked per formula in madd29 (ec29 below) and checked by
// tests/test_field29.py against a Python model.  Zero tests need a canonical
// value and are done once per bucket piece (to_fq32).
#pragma once
#include "field.cuh"
#include "f29_consts.inc"

namespace pnp {

struct F29 {
    uint32_t l[14];
};

#define F29_M 0x1FFFFFFFu

// acc + a b as ONE v_mad_u64_u32 the compiler cannot reassociate: with plain
// C++ additions LLVM starts every column's products from 0 and adds the
// carry afterwards (one v_lshl_add_u64 per column, ~5% of a product)
#ifndef PNP_F29_ASM
#define PNP_F29_ASM 0
#endif
// acc + a q with the modulus limb q in an SGPR (a compile-time constant)
__device__ __forceinline__ uint64_t mad29q(uint32_t a, uint32_t q, uint64_t acc) {
#if PNP_F29_ASM
    uint64_t r, cdummy;
    asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cdummy) : "v"(a), "s"(q), "v"(acc));
    return r;
#else
    return acc + (uint64_t)a * q;
#endif
}
__device__ __forceinline__ uint64_t mad29(uint32_t a, uint32_t b, uint64_t acc) {
#if PNP_F29_ASM
    uint64_t r, cdummy;
    asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cdummy) : "v"(a), "v"(b), "v"(acc));
    return r;
#else
    return acc + (uint64_t)a * b;
#endif
}

// Montgomery product a b 2^-406 (product scanning, one 64-bit accumulator)
__device__ __forceinline__ F29 mul29(const F29 &a, const F29 &b) {
    uint32_t m[14];
    F29 r;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 27; k++) {
#pragma unroll
        for (int i = (k > 13 ? k - 13 : 0); i <= (k < 13 ? k : 13); i++) acc = mad29(a.l[i], b.l[k - i], acc);
#pragma unroll
        for (int i = (k > 13 ? k - 13 : 0); i < (k < 14 ? k : 14); i++) acc = mad29q(m[i], F29_Q[k - i], acc);
        if (k < 14) {
            m[k] = ((uint32_t)acc * F29_QINV) & F29_M;
            acc = mad29q(m[k], F29_Q[0], acc);
        } else {
            r.l[k - 14] = (uint32_t)acc & F29_M;
        }
        acc >>= 29;
    }
    r.l[13] = (uint32_t)acc;
    return r;
}

// Montgomery square: the cross products a_i a_j (i < j) once, against the
// doubled limb 2 a_j (< 2^30): a column then holds <= 7 products < 2^59, 1
// square < 2^58 and <= 14 reduction products < 2^58 — still < 2^64.
// 105 + 196 multiply-adds instead of 196 + 196.
__device__ __forceinline__ F29 sqr29(const F29 &a) {
    uint32_t m[14], a2[14];
#pragma unroll
    for (int i = 0; i < 14; i++) a2[i] = a.l[i] << 1;
    F29 r;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 27; k++) {
#pragma unroll
        for (int i = (k > 13 ? k - 13 : 0); 2 * i < k; i++) acc = mad29(a.l[i], a2[k - i], acc);
        if ((k & 1) == 0) acc = mad29(a.l[k / 2], a.l[k / 2], acc);
#pragma unroll
        for (int i = (k > 13 ? k - 13 : 0); i < (k < 14 ? k : 14); i++) acc = mad29q(m[i], F29_Q[k - i], acc);
        if (k < 14) {
            m[k] = ((uint32_t)acc * F29_QINV) & F29_M;
            acc = mad29q(m[k], F29_Q[0], acc);
        } else {
            r.l[k - 14] = (uint32_t)acc & F29_M;
        }
        acc >>= 29;
    }
    r.l[13] = (uint32_t)acc;
    return r;
}

// a b + c d with ONE Montgomery reduction, (a b + c d) 2^-406: a column holds
// <= 14 + 14 products and <= 14 reduction products, each < 2^58, so
// < 42 * 2^58 < 2^64 with the carry; for inputs < 2^391 the result is
// < (2^783 + 2^406 q) 2^-406 < 2^382, the bound of mul29.  Saves one
// reduction (196 v_mad_u64_u32 + the column shifts) against two mul29.
__device__ __forceinline__ F29 mul2_29(const F29 &a, const F29 &b, const F29 &c, const F29 &d) {
    uint32_t m[14];
    F29 r;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 27; k++) {
#pragma unroll
        for (int i = (k > 13 ? k - 13 : 0); i <= (k < 13 ? k : 13); i++) {
            acc = mad29(a.l[i], b.l[k - i], acc);
            acc = mad29(c.l[i], d.l[k - i], acc);
        }
#pragma unroll
        for (int i = (k > 13 ? k - 13 : 0); i < (k < 14 ? k : 14); i++) acc = mad29q(m[i], F29_Q[k - i], acc);
        if (k < 14) {
            m[k] = ((uint32_t)acc * F29_QINV) & F29_M;
            acc = mad29q(m[k], F29_Q[0], acc);
        } else {
            r.l[k - 14] = (uint32_t)acc & F29_M;
        }
        acc >>= 29;
    }
    r.l[13] = (uint32_t)acc;
    return r;
}

// ---- Karatsuba forms of the a b half (round 3 A/B, tools/ubench_kara.hip).
// a = a0 + X^7 a1 (X = 2^29, 7-limb halves), likewise b:
//   a b = L + X^7 (M - L - H) + X^14 H,  L = a0 b0, H = a1 b1,
//   M = (a0 + a1)(b0 + b1)  (limb sums < 2^30: 7 products < 2^60 per column)
// 3 x 49 = 147 multiply-adds instead of 196; the column of a b at step k is
//   T_k = L_k + M_(k-7) - L_(k-7) - H_(k-7) + H_(k-14),
// assembled inside the same finely integrated Montgomery loop (the column's
// true value is >= 0 and < 2^63 whatever the order of the +/- terms, so the
// 64-bit accumulator may wrap transiently).  L_j is kept from step j to j+7,
// H_j from step j+7 to j+14.
struct KaraHalves {
    uint32_t sa[7], sb[7];
};
__device__ __forceinline__ void kara_sums(const F29 &a, const F29 &b, KaraHalves &h) {
#pragma unroll
    for (int i = 0; i < 7; i++) {
        h.sa[i] = a.l[i] + a.l[i + 7];
        h.sb[i] = b.l[i] + b.l[i + 7];
    }
}
// column j (0..12) of a 7x7 product x y, x / y given as limb pointers
#define PNP_KCOL(acc, x, y, j)                                                              \
    _Pragma("unroll") for (int i_ = ((j) > 6 ? (j) - 6 : 0); i_ <= ((j) < 6 ? (j) : 6); i_++) \
        acc = mad29((x)[i_], (y)[(j) - i_], acc)
__device__ __forceinline__ F29 mul29k(const F29 &a, const F29 &b) {
    KaraHalves h;
    kara_sums(a, b, h);
    uint32_t m[14];
    uint64_t Lk[13], Hk[13];
    F29 r;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 27; k++) {
        if (k <= 12) {
            uint64_t l = 0;
            PNP_KCOL(l, a.l, b.l, k);
            Lk[k] = l;
            acc += l;
        }
        if (k >= 7 && k <= 19) {
            const int j = k - 7;
            uint64_t hh = 0;
            PNP_KCOL(hh, a.l + 7, b.l + 7, j);
            Hk[j] = hh;
            PNP_KCOL(acc, h.sa, h.sb, j);
            acc -= Lk[j] + hh;
        }
        if (k >= 14) acc += Hk[k - 14];
#pragma unroll
        for (int i = (k > 13 ? k - 13 : 0); i < (k < 14 ? k : 14); i++) acc = mad29q(m[i], F29_Q[k - i], acc);
        if (k < 14) {
            m[k] = ((uint32_t)acc * F29_QINV) & F29_M;
            acc = mad29q(m[k], F29_Q[0], acc);
        } else {
            r.l[k - 14] = (uint32_t)acc & F29_M;
        }
        acc >>= 29;
    }
    r.l[13] = (uint32_t)acc;
    return r;
}
// a b + c d, both halves Karatsuba, one reduction (bounds as mul2_29)
__device__ __forceinline__ F29 mul2_29k(const F29 &a, const F29 &b, const F29 &c, const F29 &d) {
    KaraHalves h1, h2;
    kara_sums(a, b, h1);
    kara_sums(c, d, h2);
    uint32_t m[14];
    uint64_t Lk[13], Hk[13];
    F29 r;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 27; k++) {
        if (k <= 12) {
            uint64_t l = 0;
            PNP_KCOL(l, a.l, b.l, k);
            PNP_KCOL(l, c.l, d.l, k);
            Lk[k] = l;
            acc += l;
        }
        if (k >= 7 && k <= 19) {
            const int j = k - 7;
            uint64_t hh = 0;
            PNP_KCOL(hh, a.l + 7, b.l + 7, j);
            PNP_KCOL(hh, c.l + 7, d.l + 7, j);
            Hk[j] = hh;
            PNP_KCOL(acc, h1.sa, h1.sb, j);
            PNP_KCOL(acc, h2.sa, h2.sb, j);
            acc -= Lk[j] + hh;
        }
        if (k >= 14) acc += Hk[k - 14];
#pragma unroll
        for (int i = (k > 13 ? k - 13 : 0); i < (k < 14 ? k : 14); i++) acc = mad29q(m[i], F29_Q[k - i], acc);
        if (k < 14) {
            m[k] = ((uint32_t)acc * F29_QINV) & F29_M;
            acc = mad29q(m[k], F29_Q[0], acc);
        } else {
            r.l[k - 14] = (uint32_t)acc & F29_M;
        }
        acc >>= 29;
    }
    r.l[13] = (uint32_t)acc;
    return r;
}
#undef PNP_KCOL

// a + K - b (K = F29_KA or F29_KB, b < K), carries normalised
__device__ __forceinline__ F29 sub29(const F29 &a, const F29 &b, const uint32_t *K) {
    F29 r;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 13; i++) {
        uint32_t t = a.l[i] + K[i] - b.l[i] + c;
        r.l[i] = t & F29_M;
        c = t >> 29;
    }
    r.l[13] = a.l[13] + K[13] - b.l[13] + c;
    return r;
}

// K - b
__device__ __forceinline__ F29 neg29(const F29 &b, const uint32_t *K) {
    F29 r;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 13; i++) {
        uint32_t t = K[i] - b.l[i] + c;
        r.l[i] = t & F29_M;
        c = t >> 29;
    }
    r.l[13] = K[13] - b.l[13] + c;
    return r;
}

__device__ __forceinline__ F29 const29(const uint32_t *c) {
    F29 r;
#pragma unroll
    for (int i = 0; i < 14; i++) r.l[i] = c[i];
    return r;
}

// 12 x 32-bit limbs -> 14 x 29-bit limbs (same integer)
__device__ __forceinline__ F29 repack29(const uint32_t *v) {
    F29 r;
#pragma unroll
    for (int j = 0; j < 14; j++) {
        const int bit = 29 * j, w = bit >> 5, sh = bit & 31;
        uint64_t x = v[w];
        if (w + 1 < 12) x |= (uint64_t)v[w + 1] << 32;
        r.l[j] = (uint32_t)(x >> sh) & F29_M;
    }
    return r;
}

// integer < 2q (limbs normalised, < 2^384) -> canonical Fq (12 x 32-bit limbs)
__device__ __forceinline__ Fq unpack29(const F29 &a) {
    Fq r;
#pragma unroll
    for (int w = 0; w < 12; w++) {
        const int bit = 32 * w, j = bit / 29, sh = bit % 29;
        uint64_t x = (uint64_t)a.l[j] >> sh;
        if (j + 1 < 14) x |= (uint64_t)a.l[j + 1] << (29 - sh);
        if (j + 2 < 14 && 58 - sh < 32) x |= (uint64_t)a.l[j + 2] << (58 - sh);
        r.v[w] = (uint32_t)x;
    }
    reduce_once(r);
    return r;
}

// R406-form F29 -> R384-form canonical Fq
__device__ __forceinline__ Fq to_fq32(const F29 &a) { return unpack29(mul29(a, const29(F29_C384))); }
// R384-form Fq (canonical) -> R406-form F29 (< 2q)
__device__ __forceinline__ F29 from_fq32(const Fq &a) { return mul29(repack29(a.v), const29(F29_C428)); }

}  // namespace pnp
