// fr29.cuh — BLS12-381 Fr in radix 2^29 (nine limbs) for the NTT passes on
// gfx950.
//
// Why: the 32-bit-limb product (field.cuh) pairs every v_mad_u64_u32 with a
// v_addc_co_u32 to carry the column sums, and its add / sub / select chains run
// through VCC with wait states between the links.  With 29-bit limbs a column
// (<= 9 products + 9 reduction products + carry) fits one 64-bit accumulator:
// the product is 162 bare v_mad_u64_u32 plus one shift / mask per column, and
// sums / differences carry by shift and mask in ordinary VGPRs.
//
// Representation: value = sum l_i 2^(29 i), l_0..l_7 < 2^29, the top limb
// l_8 < 2^32 holds everything above bit 232 (values < 2^264).  The data keep
// the HBM form's Montgomery factor (2^256, field.cuh); twiddles and twist
// factors are stored times 2^261 (tables built by ntt.hip), so r29_mul
// (x y 2^-261) maps data to data.  Nothing is reduced inside a pass: a DIF
// level doubles the bound (a + b), a difference adds a multiple of r with
// lifted limbs (no borrows), a product is < x y / 2^261 + r; r29_canon brings
// a pass's outputs (< 2^264) back to [0, r).  tests/test_fr29.py models every
// operation limb for limb with the bounds asserted.
#pragma once
#include "field.cuh"
#include "fr29_consts.inc"

namespace pnp {

struct R29 {
    uint32_t l[9];
};

#define R29_M 0x1FFFFFFFu

// 8 x 32-bit words (any value < 2^256) -> nine limbs, same integer
__device__ __forceinline__ R29 r29_from_words(const uint32_t *v) {
    R29 r;
#pragma unroll
    for (int j = 0; j < 9; j++) {
        const int bit = 29 * j, w = bit >> 5, sh = bit & 31;
        uint32_t x = v[w] >> sh;
        if (sh > 3 && w + 1 < 8) x |= v[w + 1] << (32 - sh);
        r.l[j] = j < 8 ? (x & R29_M) : x;
    }
    return r;
}

// value < 2^256 (canonical after r29_canon) -> 8 x 32-bit words
__device__ __forceinline__ void r29_to_words(const R29 &a, uint32_t *v) {
#pragma unroll
    for (int w = 0; w < 8; w++) {
        const int bit = 32 * w, j = bit / 29, sh = bit % 29;
        uint32_t x = a.l[j] >> sh;
        if (j + 1 < 9) x |= a.l[j + 1] << (29 - sh);
        if (j + 2 < 9 && 58 - sh < 32) x |= a.l[j + 2] << (58 - sh);
        v[w] = x;
    }
}

__device__ __forceinline__ R29 r29_add(const R29 &a, const R29 &b) {
    R29 r;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint32_t t = a.l[i] + b.l[i] + c;
        r.l[i] = t & R29_M;
        c = t >> 29;
    }
    r.l[8] = a.l[8] + b.l[8] + c;
    return r;
}

// a + K - b, K a limb-lifted multiple of r larger than b
__device__ __forceinline__ R29 r29_sub(const R29 &a, const R29 &b, const uint32_t *K) {
    R29 r;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint32_t t = a.l[i] + K[i] - b.l[i] + c;
        r.l[i] = t & R29_M;
        c = t >> 29;
    }
    r.l[8] = a.l[8] + K[8] - b.l[8] + c;
    return r;
}

// a b 2^-261 (mod r, < a b / 2^261 + r); r = 1 mod 2^29, so the Montgomery
// digit is -acc mod 2^29 and its product with r_0 is the digit itself
__device__ __forceinline__ R29 r29_mul(const R29 &a, const R29 &b) {
    uint32_t m[9];
    R29 r;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 17; k++) {
#pragma unroll
        for (int i = (k > 8 ? k - 8 : 0); i <= (k < 8 ? k : 8); i++) acc += (uint64_t)a.l[i] * b.l[k - i];
#pragma unroll
        for (int i = (k > 8 ? k - 8 : 0); i < (k < 9 ? k : 9); i++) acc += (uint64_t)m[i] * R29_P[k - i];
        if (k < 9) {
            m[k] = (0u - (uint32_t)acc) & R29_M;
            acc += m[k];
        } else {
            r.l[k - 9] = (uint32_t)acc & R29_M;
        }
        acc >>= 29;
    }
    r.l[8] = (uint32_t)acc;
    return r;
}

// (a b + c d) 2^-261 with one reduction (< (a b + c d) / 2^261 + r); every
// column holds <= 27 products of normalised limbs (< 2^58 each): < 2^63
__device__ __forceinline__ R29 r29_mul2(const R29 &a, const R29 &b, const R29 &c, const R29 &d) {
    uint32_t m[9];
    R29 r;
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 17; k++) {
#pragma unroll
        for (int i = (k > 8 ? k - 8 : 0); i <= (k < 8 ? k : 8); i++) {
            acc += (uint64_t)a.l[i] * b.l[k - i];
            acc += (uint64_t)c.l[i] * d.l[k - i];
        }
#pragma unroll
        for (int i = (k > 8 ? k - 8 : 0); i < (k < 9 ? k : 9); i++) acc += (uint64_t)m[i] * R29_P[k - i];
        if (k < 9) {
            m[k] = (0u - (uint32_t)acc) & R29_M;
            acc += m[k];
        } else {
            r.l[k - 9] = (uint32_t)acc & R29_M;
        }
        acc >>= 29;
    }
    r.l[8] = (uint32_t)acc;
    return r;
}

// x < 2^264 -> x mod r: q = floor(l_8 MU / 2^32) <= x / r falls short of it by
// at most 2, x - q r = x + q (2^261 - r) - q 2^261, then two conditional
// subtractions of r (y >= r iff y + 2^261 - r reaches bit 261)
__device__ __forceinline__ R29 r29_canon(const R29 &x) {
    const uint32_t q = (uint32_t)(((uint64_t)x.l[8] * R29_MU) >> 32);
    R29 y;
    uint64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        acc += x.l[i] + (uint64_t)q * R29_C[i];
        y.l[i] = (uint32_t)acc & R29_M;
        acc >>= 29;
    }
    y.l[8] = (uint32_t)(acc + x.l[8] + (uint64_t)q * R29_C[8] - ((uint64_t)q << 29));
#pragma unroll
    for (int rep = 0; rep < 2; rep++) {
        R29 z;
        uint32_t c = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t t = y.l[i] + R29_C[i] + c;
            z.l[i] = t & R29_M;
            c = t >> 29;
        }
        const uint32_t t = y.l[8] + R29_C[8] + c;
        const bool ge = t >= (1u << 29);
        z.l[8] = t - (1u << 29);
#pragma unroll
        for (int i = 0; i < 9; i++) y.l[i] = ge ? z.l[i] : y.l[i];
    }
    return y;
}

// tables of 2^261-form factors: 9 u32 per entry
__device__ __forceinline__ R29 r29_load(const uint32_t *t, uint64_t i) {
    const uint32_t *p = t + 9 * i;
    R29 r;
#pragma unroll
    for (int k = 0; k < 9; k++) r.l[k] = p[k];
    return r;
}

}  // namespace pnp
