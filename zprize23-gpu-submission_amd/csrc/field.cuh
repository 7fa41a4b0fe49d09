// field.cuh — BLS12-381 Fr / Fq Montgomery arithmetic for gfx950 (and host).
//
// Semantics restated from lib/PLONK/utils/mont/cuda/ff/mont_t.cuh (Montgomery
// form, R = 2^256 / 2^384, fully reduced residues) with the constants of
// ff/bls12-381.hpp:7-93.  The implementation is CDNA-first: 32-bit limbs so the
// inner products map to v_mad_u64_u32 (32x32+64 -> 64, one VALU op per limb
// product), carry chains through 64-bit adds (v_add_co / v_addc_co), and the
// "no-carry" CIOS variant, valid because both moduli leave the top bit of the
// top 32-bit word clear (r: 0x73eda753.., q: 0x1a0111ea..).  An element is 8 /
// 12 VGPRs; memory layout equals the reference's 4 / 6 little-endian u64 limbs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PNP_HD __host__ __device__ __forceinline__
#define PNP_LIMB(x) (uint32_t)(x##ULL), (uint32_t)(x##ULL >> 32)

namespace pnp {

struct FrP {
    static constexpr int N = 8;
    static constexpr uint32_t INV = 0xffffffffu;  // -r^-1 mod 2^32
    static constexpr uint32_t P[8] = {PNP_LIMB(0xffffffff00000001), PNP_LIMB(0x53bda402fffe5bfe),
                                      PNP_LIMB(0x3339d80809a1d805), PNP_LIMB(0x73eda753299d7d48)};
    static constexpr uint32_t ONE[8] = {PNP_LIMB(0x00000001fffffffe), PNP_LIMB(0x5884b7fa00034802),
                                        PNP_LIMB(0x998c4fefecbc4ff5), PNP_LIMB(0x1824b159acc5056f)};
    static constexpr uint32_t R2[8] = {PNP_LIMB(0xc999e990f3f29c6d), PNP_LIMB(0x2b6cedcb87925c23),
                                       PNP_LIMB(0x05d314967254398f), PNP_LIMB(0x0748d9d99f59ff11)};
    // r - 2 (Fermat exponent)
    static constexpr uint32_t PM2[8] = {PNP_LIMB(0xfffffffeffffffff), PNP_LIMB(0x53bda402fffe5bfe),
                                        PNP_LIMB(0x3339d80809a1d805), PNP_LIMB(0x73eda753299d7d48)};
};

struct FqP {
    static constexpr int N = 12;
    static constexpr uint32_t INV = 0xfffcfffdu;  // -q^-1 mod 2^32
    static constexpr uint32_t P[12] = {PNP_LIMB(0xb9feffffffffaaab), PNP_LIMB(0x1eabfffeb153ffff),
                                       PNP_LIMB(0x6730d2a0f6b0f624), PNP_LIMB(0x64774b84f38512bf),
                                       PNP_LIMB(0x4b1ba7b6434bacd7), PNP_LIMB(0x1a0111ea397fe69a)};
    static constexpr uint32_t ONE[12] = {PNP_LIMB(0x760900000002fffd), PNP_LIMB(0xebf4000bc40c0002),
                                         PNP_LIMB(0x5f48985753c758ba), PNP_LIMB(0x77ce585370525745),
                                         PNP_LIMB(0x5c071a97a256ec6d), PNP_LIMB(0x15f65ec3fa80e493)};
    static constexpr uint32_t R2[12] = {PNP_LIMB(0xf4df1f341c341746), PNP_LIMB(0x0a76e6a609d104f1),
                                        PNP_LIMB(0x8de5476c4c95b6d5), PNP_LIMB(0x67eb88a9939d83c0),
                                        PNP_LIMB(0x9a793e85b519952d), PNP_LIMB(0x11988fe592cae3aa)};
    static constexpr uint32_t PM2[12] = {PNP_LIMB(0xb9feffffffffaaa9), PNP_LIMB(0x1eabfffeb153ffff),
                                         PNP_LIMB(0x6730d2a0f6b0f624), PNP_LIMB(0x64774b84f38512bf),
                                         PNP_LIMB(0x4b1ba7b6434bacd7), PNP_LIMB(0x1a0111ea397fe69a)};
};

template <class P>
struct Fp {
    static constexpr int N = P::N;
    uint32_t v[N];

    PNP_HD static Fp zero() {
        Fp r;
#pragma unroll
        for (int i = 0; i < N; i++) r.v[i] = 0;
        return r;
    }
    PNP_HD static Fp one() {
        Fp r;
#pragma unroll
        for (int i = 0; i < N; i++) r.v[i] = P::ONE[i];
        return r;
    }
    PNP_HD static Fp r2() {
        Fp r;
#pragma unroll
        for (int i = 0; i < N; i++) r.v[i] = P::R2[i];
        return r;
    }
    PNP_HD static Fp modulus() {
        Fp r;
#pragma unroll
        for (int i = 0; i < N; i++) r.v[i] = P::P[i];
        return r;
    }
    PNP_HD bool is_zero() const {
        uint32_t acc = 0;
#pragma unroll
        for (int i = 0; i < N; i++) acc |= v[i];
        return acc == 0;
    }
    PNP_HD bool operator==(const Fp &o) const {
        uint32_t acc = 0;
#pragma unroll
        for (int i = 0; i < N; i++) acc |= v[i] ^ o.v[i];
        return acc == 0;
    }
    PNP_HD bool operator!=(const Fp &o) const { return !(*this == o); }
};

using Fr = Fp<FrP>;
using Fq = Fp<FqP>;

// ---- raw multi-limb helpers ----
// On the device the carry chains use clang's add/sub-with-carry builtins,
// which lower to one v_add_co_u32 / v_addc_co_u32 (v_sub_co / v_subb_co) per
// limb.  The 64-bit formulation below compiled to two v_lshl_add_u64 and
// three v_mov per limb (measured: a fifth of an NTT butterfly's VALU issue).
template <int N>
PNP_HD uint32_t add_n(uint32_t *r, const uint32_t *a, const uint32_t *b) {
#ifdef __HIP_DEVICE_COMPILE__
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < N; i++) r[i] = __builtin_addc(a[i], b[i], c, &c);
    return c;
#else
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < N; i++) {
        c = (uint64_t)a[i] + b[i] + (c >> 32);
        r[i] = (uint32_t)c;
    }
    return (uint32_t)(c >> 32);
#endif
}
template <int N>
PNP_HD uint32_t sub_n(uint32_t *r, const uint32_t *a, const uint32_t *b) {
#ifdef __HIP_DEVICE_COMPILE__
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < N; i++) r[i] = __builtin_subc(a[i], b[i], br, &br);
    return br;
#else
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < N; i++) {
        uint64_t d = (uint64_t)a[i] - b[i] - br;
        r[i] = (uint32_t)d;
        br = (uint32_t)(d >> 32) & 1u;
    }
    return br;
#endif
}

// r = a - P if a >= P else a   (a < 2P)
template <class P>
PNP_HD void reduce_once(Fp<P> &a) {
    constexpr int N = P::N;
    uint32_t t[N];
    uint32_t br = sub_n<N>(t, a.v, P::P);
#pragma unroll
    for (int i = 0; i < N; i++) a.v[i] = br ? a.v[i] : t[i];
}

template <class P>
PNP_HD Fp<P> operator+(const Fp<P> &a, const Fp<P> &b) {
    Fp<P> r;
    add_n<P::N>(r.v, a.v, b.v);  // < 2P < 2^(32N): no carry out for both moduli
    reduce_once(r);
    return r;
}
template <class P>
PNP_HD Fp<P> operator-(const Fp<P> &a, const Fp<P> &b) {
    constexpr int N = P::N;
    Fp<P> r;
    uint32_t br = sub_n<N>(r.v, a.v, b.v);
    uint32_t t[N];
    add_n<N>(t, r.v, P::P);
#pragma unroll
    for (int i = 0; i < N; i++) r.v[i] = br ? t[i] : r.v[i];
    return r;
}
template <class P>
PNP_HD Fp<P> neg(const Fp<P> &a) {
    return Fp<P>::zero() - a;
}
template <class P>
PNP_HD Fp<P> dbl(const Fp<P> &a) {
    return a + a;
}

#ifdef __HIP_DEVICE_COMPILE__
// One limb product accumulated into a 96-bit column accumulator (acc2:acc):
// v_mad_u64_u32 writes its 64-bit carry-out to VCC, v_addc_co_u32 folds it
// into the third word.  Measured on gfx950: v_mad_u64_u32 is half rate, the
// same as v_mul_lo_u32 or a 64-bit add, so two instructions per product is
// the floor for 32-bit limbs.
__device__ __forceinline__ void mac96(uint64_t &acc, uint32_t &acc2, uint32_t a, uint32_t b) {
    asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32 %1, vcc, 0, %1, vcc"
        : "+v"(acc), "+v"(acc2)
        : "v"(a), "v"(b)
        : "vcc");
}

// a*b and m*p into the same column in one asm block (halves the hazard
// s_nop the compiler places after every opaque asm statement)
__device__ __forceinline__ void mac96x2(uint64_t &acc, uint32_t &acc2, uint32_t a, uint32_t b,
                                        uint32_t m, uint32_t p) {
    asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\t"
        "v_addc_co_u32 %1, vcc, 0, %1, vcc\n\t"
        "v_mad_u64_u32 %0, vcc, %4, %5, %0\n\t"
        "v_addc_co_u32 %1, vcc, 0, %1, vcc"
        : "+v"(acc), "+v"(acc2)
        : "v"(a), "v"(b), "v"(m), "s"(p)
        : "vcc");
}

// Montgomery product by finely-integrated product scanning (FIPS): column k
// of a*b and of m*p are summed into one 96-bit accumulator; m_k is chosen so
// the low word of column k (k < N) vanishes; columns N..2N-1 are the result.
// 2N^2 (mad + addc) + N mul_lo + ~3 movs per column, no CIOS temporaries.
//   PNP_MONT_VARIANT 0 : one asm statement per product pair (compiler pads
//                        each statement with an s_nop)
//   PNP_MONT_VARIANT 1 : the whole product as one asm block, one chain
//   PNP_MONT_VARIANT 2 : one block, a*b and m*p on two independent chains
#ifndef PNP_MONT_VARIANT
#define PNP_MONT_VARIANT 0
#endif
#include "mont_asm.inc"
// REDUCE = false: the result is left in [0, 2P) (no final conditional
// subtraction); valid for a b < R P, e.g. a < 4P, b < P for Fr (4r < 2^256)
template <class P, bool REDUCE = true>
__device__ __forceinline__ Fp<P> mont_mul_dev(const Fp<P> &a, const Fp<P> &b) {
    constexpr int N = P::N;
    Fp<P> r;
#if PNP_MONT_VARIANT == 1 || PNP_MONT_VARIANT == 2
    uint32_t p[N];
#pragma unroll
    for (int i = 0; i < N; i++) p[i] = P::P[i];
    if constexpr (N == 12) {
#if PNP_MONT_VARIANT == 1
        mont_asm12_single(r.v, a.v, b.v, p, P::INV);
#else
        mont_asm12_dual(r.v, a.v, b.v, p, P::INV);
#endif
    } else {
        static_assert(N == 8 && P::INV == 0xffffffffu, "Fr expected");
#if PNP_MONT_VARIANT == 1
        mont_asm8_single(r.v, a.v, b.v, p);
#else
        mont_asm8_dual(r.v, a.v, b.v, p);
#endif
    }
#else
    uint32_t m[N];
    uint64_t acc = 0;
    uint32_t acc2 = 0;
#pragma unroll
    for (int k = 0; k < N; k++) {
#pragma unroll
        for (int j = 0; j < k; j++) mac96x2(acc, acc2, a.v[j], b.v[k - j], m[j], P::P[k - j]);
        mac96(acc, acc2, a.v[k], b.v[0]);
        m[k] = (uint32_t)acc * P::INV;
        mac96(acc, acc2, m[k], P::P[0]);
        acc = (acc >> 32) | ((uint64_t)acc2 << 32);
        acc2 = 0;
    }
#pragma unroll
    for (int k = N; k < 2 * N; k++) {
#pragma unroll
        for (int j = k - N + 1; j < N; j++) mac96x2(acc, acc2, a.v[j], b.v[k - j], m[j], P::P[k - j]);
        r.v[k - N] = (uint32_t)acc;
        acc = (acc >> 32) | ((uint64_t)acc2 << 32);
        acc2 = 0;
    }
#endif
    if (REDUCE) reduce_once(r);  // result < 2P < 2^(32N) for both moduli
    return r;
}

// a b + c d with ONE Montgomery reduction (same product scanning; a column
// now sums up to 3N products, still < 2^96).  For Fr: (a b + c d + m r) 2^-256
// < r (2 r / 2^256 + 1) < 2r, so one conditional subtraction leaves it
// canonical.  Saves a reduction and a modular addition against two products.
__device__ __forceinline__ Fr mont_mul2_dev(const Fr &a, const Fr &b, const Fr &c, const Fr &d) {
    constexpr int N = FrP::N;
    Fr r;
    uint32_t m[N];
    uint64_t acc = 0;
    uint32_t acc2 = 0;
#pragma unroll
    for (int k = 0; k < N; k++) {
#pragma unroll
        for (int j = 0; j < k; j++) {
            mac96x2(acc, acc2, a.v[j], b.v[k - j], m[j], FrP::P[k - j]);
            mac96(acc, acc2, c.v[j], d.v[k - j]);
        }
        mac96(acc, acc2, a.v[k], b.v[0]);
        mac96(acc, acc2, c.v[k], d.v[0]);
        m[k] = (uint32_t)acc * FrP::INV;
        mac96(acc, acc2, m[k], FrP::P[0]);
        acc = (acc >> 32) | ((uint64_t)acc2 << 32);
        acc2 = 0;
    }
#pragma unroll
    for (int k = N; k < 2 * N; k++) {
#pragma unroll
        for (int j = k - N + 1; j < N; j++) {
            mac96x2(acc, acc2, a.v[j], b.v[k - j], m[j], FrP::P[k - j]);
            mac96(acc, acc2, c.v[j], d.v[k - j]);
        }
        r.v[k - N] = (uint32_t)acc;
        acc = (acc >> 32) | ((uint64_t)acc2 << 32);
        acc2 = 0;
    }
    reduce_once(r);
    return r;
}
#endif

#ifndef __HIP_DEVICE_COMPILE__
// Host Montgomery product: CIOS on 64-bit words with 128-bit products (the
// x86-64 mul gives the full 64x64 product).  The prover's host work between
// device round trips (challenge arithmetic, the commitments' affine
// conversion) sits on the proof's critical path: the 32-bit-limb form below
// cost 121 ns per Fr product, 185 us per Fq inversion.
template <class P>
constexpr uint64_t mont_inv64() {  // -P^-1 mod 2^64 (Newton: each step doubles the bits)
    const uint64_t p0 = (uint64_t)P::P[0] | (uint64_t)P::P[1] << 32;
    uint64_t x = 1;
    for (int i = 0; i < 7; i++) x *= 2 - p0 * x;
    return 0 - x;
}
template <class P>
inline Fp<P> mont_mul_host(const Fp<P> &a, const Fp<P> &b) {
    constexpr int M = P::N / 2;
    constexpr uint64_t INV = mont_inv64<P>();
    typedef unsigned __int128 u128;
    uint64_t A[M], B[M], Q[M], t[M + 2];
#pragma unroll
    for (int j = 0; j < M; j++) {
        A[j] = (uint64_t)a.v[2 * j] | (uint64_t)a.v[2 * j + 1] << 32;
        B[j] = (uint64_t)b.v[2 * j] | (uint64_t)b.v[2 * j + 1] << 32;
        Q[j] = (uint64_t)P::P[2 * j] | (uint64_t)P::P[2 * j + 1] << 32;
        t[j] = 0;
    }
    t[M] = t[M + 1] = 0;
#pragma unroll
    for (int i = 0; i < M; i++) {
        u128 c = 0;
#pragma unroll
        for (int j = 0; j < M; j++) {
            c = (u128)A[j] * B[i] + t[j] + (uint64_t)(c >> 64);
            t[j] = (uint64_t)c;
        }
        c = (u128)t[M] + (uint64_t)(c >> 64);
        t[M] = (uint64_t)c;
        t[M + 1] = (uint64_t)(c >> 64);
        const uint64_t m = t[0] * INV;
        c = (u128)m * Q[0] + t[0];
#pragma unroll
        for (int j = 1; j < M; j++) {
            c = (u128)m * Q[j] + t[j] + (uint64_t)(c >> 64);
            t[j - 1] = (uint64_t)c;
        }
        c = (u128)t[M] + (uint64_t)(c >> 64);
        t[M - 1] = (uint64_t)c;
        t[M] = t[M + 1] + (uint64_t)(c >> 64);
    }
    // CIOS leaves [0, 2P) (t[M] = 0 for a, b < P < R / 4): one conditional
    // subtraction, on the 64-bit words
    uint64_t d[M], br = 0;
#pragma unroll
    for (int j = 0; j < M; j++) {
        const u128 x = (u128)t[j] - Q[j] - br;
        d[j] = (uint64_t)x;
        br = (uint64_t)(x >> 64) & 1;
    }
    Fp<P> r;
#pragma unroll
    for (int j = 0; j < M; j++) {
        const uint64_t w = br ? t[j] : d[j];
        r.v[2 * j] = (uint32_t)w;
        r.v[2 * j + 1] = (uint32_t)(w >> 32);
    }
    return r;
}
#endif

// Montgomery product: mont_mul_dev on the device, mont_mul_host on the host.
// (The "no-carry" CIOS on 32-bit limbs after the return was the host path;
// it is kept only for host builds without a 128-bit integer type.)
template <class P>
PNP_HD Fp<P> operator*(const Fp<P> &a, const Fp<P> &b) {
#ifdef __HIP_DEVICE_COMPILE__
    return mont_mul_dev(a, b);
#elif defined(__SIZEOF_INT128__)
    return mont_mul_host(a, b);
#endif
    constexpr int N = P::N;
    uint32_t t[N];
#pragma unroll
    for (int j = 0; j < N; j++) t[j] = 0;
#pragma unroll
    for (int i = 0; i < N; i++) {
        uint64_t A = (uint64_t)a.v[0] * b.v[i] + t[0];
        t[0] = (uint32_t)A;
        uint32_t m = t[0] * P::INV;
        uint64_t C = (uint64_t)m * P::P[0] + t[0];
#pragma unroll
        for (int j = 1; j < N; j++) {
            A = (uint64_t)a.v[j] * b.v[i] + t[j] + (A >> 32);
            t[j] = (uint32_t)A;
            C = (uint64_t)m * P::P[j] + t[j] + (C >> 32);
            t[j - 1] = (uint32_t)C;
        }
        t[N - 1] = (uint32_t)(A >> 32) + (uint32_t)(C >> 32);
    }
    Fp<P> r;
#pragma unroll
    for (int j = 0; j < N; j++) r.v[j] = t[j];
    reduce_once(r);
    return r;
}
template <class P>
PNP_HD Fp<P> sqr(const Fp<P> &a) {
    return a * a;
}
// a b + c d (one Montgomery reduction on the device, mont_mul2_dev)
PNP_HD Fr fr_mul2(const Fr &a, const Fr &b, const Fr &c, const Fr &d) {
#ifdef __HIP_DEVICE_COMPILE__
    return mont_mul2_dev(a, b, c, d);
#else
    return a * b + c * d;
#endif
}

// Out-of-line Fq product for the EC formulas: one copy of the 288-mad body
// per kernel instead of 10-18 inlined copies per point operation (inlining
// all of them made LLVM's scheduler take 30-40 min per translation unit).
#ifdef __HIP_DEVICE_COMPILE__
__device__ __noinline__ Fq fq_mul_ool(Fq a, Fq b);
#endif
PNP_HD Fq fq_mul(const Fq &a, const Fq &b) {
#if defined(__HIP_DEVICE_COMPILE__) && defined(PNP_FQ_OUTLINE)
    return fq_mul_ool(a, b);
#else
    return a * b;
#endif
}

template <class P>
PNP_HD Fp<P> &operator+=(Fp<P> &a, const Fp<P> &b) { return a = a + b; }
template <class P>
PNP_HD Fp<P> &operator-=(Fp<P> &a, const Fp<P> &b) { return a = a - b; }
template <class P>
PNP_HD Fp<P> &operator*=(Fp<P> &a, const Fp<P> &b) { return a = a * b; }

template <class P>
PNP_HD Fp<P> to_mont(const Fp<P> &a) { return a * Fp<P>::r2(); }
template <class P>
PNP_HD Fp<P> from_mont(const Fp<P> &a) {
    Fp<P> one_raw = Fp<P>::zero();
    one_raw.v[0] = 1;
    return a * one_raw;
}

// x^e for a small exponent (exp_mod_kernel_, mont_arithmetic.cu:89)
template <class P>
PNP_HD Fp<P> pow_u64(Fp<P> base, uint64_t e) {
    Fp<P> acc = Fp<P>::one();
    while (e) {
        if (e & 1) acc = acc * base;
        base = base * base;
        e >>= 1;
    }
    return acc;
}

#ifndef __HIP_DEVICE_COMPILE__
// Host inverse by the binary extended Euclidean algorithm on 64-bit words
// (~2 log2 P shift / subtract steps instead of Fermat's ~1.5 log2 P dependent
// products: an Fq inverse in a few us, not ~65).  The host inverts public
// values only (challenge arithmetic, the commitments' affine conversion), so
// its data-dependent time leaks nothing.  Montgomery form in and out: the
// plain inverse of aR is a^-1 R^-1, and one product by R^3 gives a^-1 R.
template <class P>
inline Fp<P> inverse_host(const Fp<P> &a) {
    constexpr int M = P::N / 2;
    typedef unsigned __int128 u128;
    if (a.is_zero()) return a;
    uint64_t u[M], v[M], x1[M], x2[M], q[M];
    for (int j = 0; j < M; j++) {
        u[j] = (uint64_t)a.v[2 * j] | (uint64_t)a.v[2 * j + 1] << 32;
        q[j] = v[j] = (uint64_t)P::P[2 * j] | (uint64_t)P::P[2 * j + 1] << 32;
        x1[j] = x2[j] = 0;
    }
    x1[0] = 1;
    auto is_one = [](const uint64_t *w) {
        uint64_t acc = w[0] ^ 1;
        for (int j = 1; j < M; j++) acc |= w[j];
        return acc == 0;
    };
    auto shr1 = [](uint64_t *w, uint64_t top) {  // w = (top:w) >> 1
        for (int j = 0; j < M - 1; j++) w[j] = (w[j] >> 1) | (w[j + 1] << 63);
        w[M - 1] = (w[M - 1] >> 1) | (top << 63);
    };
    auto halve = [&](uint64_t *x) {  // x / 2 mod P (x < P)
        uint64_t c = 0;
        if (x[0] & 1) {
            u128 t = 0;
            for (int j = 0; j < M; j++) {
                t = (u128)x[j] + q[j] + (uint64_t)(t >> 64);
                x[j] = (uint64_t)t;
            }
            c = (uint64_t)(t >> 64);
        }
        shr1(x, c);
    };
    auto sub = [](uint64_t *r, const uint64_t *b) {  // r -= b, borrow out
        uint64_t br = 0;
        for (int j = 0; j < M; j++) {
            const u128 t = (u128)r[j] - b[j] - br;
            r[j] = (uint64_t)t;
            br = (uint64_t)(t >> 64) & 1;
        }
        return br;
    };
    auto geq = [](const uint64_t *x, const uint64_t *y) {
        for (int j = M - 1; j >= 0; j--)
            if (x[j] != y[j]) return x[j] > y[j];
        return true;
    };
    auto sub_mod = [&](uint64_t *r, const uint64_t *b) {  // r = r - b mod P
        if (sub(r, b)) {
            u128 t = 0;
            for (int j = 0; j < M; j++) {
                t = (u128)r[j] + q[j] + (uint64_t)(t >> 64);
                r[j] = (uint64_t)t;
            }
        }
    };
    while (!is_one(u) && !is_one(v)) {
        while (!(u[0] & 1)) {
            shr1(u, 0);
            halve(x1);
        }
        while (!(v[0] & 1)) {
            shr1(v, 0);
            halve(x2);
        }
        if (geq(u, v)) {
            sub(u, v);
            sub_mod(x1, x2);
        } else {
            sub(v, u);
            sub_mod(x2, x1);
        }
    }
    const uint64_t *x = is_one(u) ? x1 : x2;
    Fp<P> r;
    for (int j = 0; j < M; j++) {
        r.v[2 * j] = (uint32_t)x[j];
        r.v[2 * j + 1] = (uint32_t)(x[j] >> 32);
    }
    const Fp<P> r3 = mont_mul_host(Fp<P>::r2(), Fp<P>::r2());  // R^3 mod P
    return mont_mul_host(r, r3);
}
#endif

// Fermat inverse a^(P-2); inv(0) = 0 (inv_mod_kernel_, mont_arithmetic.cu:73).
// The host takes inverse_host above.
template <class P>
PNP_HD Fp<P> inverse(const Fp<P> &a) {
#if !defined(__HIP_DEVICE_COMPILE__) && defined(__SIZEOF_INT128__)
    return inverse_host(a);
#endif
    Fp<P> acc = Fp<P>::one();
    for (int w = P::N - 1; w >= 0; w--) {
        uint32_t e = P::PM2[w];
        for (int b = 31; b >= 0; b--) {
            acc = acc * acc;
            if ((e >> b) & 1) acc = acc * a;
        }
    }
    return acc;
}

// Fr inverse by the binary extended Euclidean algorithm on 32-bit words, for
// the device where ONE inversion's latency is the cost (the batch inverse's
// base case, poly.hip k_inv_small): ~2 log2 r steps of a few 8-word shifts /
// subtractions instead of Fermat's ~380 dependent products of ~300 VALU.
// Variable time; it inverts the product of a batch, not a key.  Halving x
// (mod r) by 2^k at once: r = 1 mod 2^32, so x + ((-x) mod 2^k) r is
// divisible by 2^k.
PNP_HD void inv_shr(uint32_t *w, int k) {  // w >>= k, 0 < k < 32
#pragma unroll
    for (int j = 0; j < 7; j++) w[j] = (w[j] >> k) | (w[j + 1] << (32 - k));
    w[7] >>= k;
}
PNP_HD void inv_halve(uint32_t *x, int k) {  // x 2^-k mod r (x < r), 0 < k < 32
    const uint32_t m = (0u - x[0]) & ((1u << k) - 1);
    uint64_t c = 0;
    uint32_t top;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        c += (uint64_t)m * FrP::P[j] + x[j];
        x[j] = (uint32_t)c;
        c >>= 32;
    }
    top = (uint32_t)c;  // x + m r < 2^(256 + k)
#pragma unroll
    for (int j = 0; j < 7; j++) x[j] = (x[j] >> k) | (x[j + 1] << (32 - k));
    x[7] = (x[7] >> k) | (top << (32 - k));
    // (x + m r) / 2^k < r / 2^k + r: one conditional subtraction
    uint32_t t[8], br = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) t[j] = __builtin_subc(x[j], FrP::P[j], br, &br);
#pragma unroll
    for (int j = 0; j < 8; j++) x[j] = br ? x[j] : t[j];
}
PNP_HD Fr fr_inverse_bin(const Fr &a) {
    if (a.is_zero()) return a;
    uint32_t u[8], v[8], x1[8], x2[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
        u[j] = a.v[j];
        v[j] = FrP::P[j];
        x1[j] = x2[j] = 0;
    }
    x1[0] = 1;
    auto is_one = [](const uint32_t *w) {
        uint32_t acc = w[0] ^ 1u;
#pragma unroll
        for (int j = 1; j < 8; j++) acc |= w[j];
        return acc == 0;
    };
    auto strip = [](uint32_t *w, uint32_t *x) {  // w odd, x / 2^k (w != 0)
        while (!(w[0] & 1)) {
            const int k = w[0] ? __builtin_ctz(w[0]) : 31;
            inv_shr(w, k);
            inv_halve(x, k);
        }
    };
    strip(u, x1);
    while (!is_one(u) && !is_one(v)) {
        strip(v, x2);
        bool ge = true;  // u >= v
#pragma unroll
        for (int j = 7; j >= 0; j--)
            if (u[j] != v[j]) {
                ge = u[j] > v[j];
                break;
            }
        // keep u >= v: swapping the pairs (u, x1), (v, x2) keeps x1 a = u,
        // x2 a = v (mod r); selects, not pointers (registers, no scratch)
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t tu = u[j], tx = x1[j];
            u[j] = ge ? tu : v[j];
            v[j] = ge ? v[j] : tu;
            x1[j] = ge ? tx : x2[j];
            x2[j] = ge ? x2[j] : tx;
        }
        uint32_t br = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) u[j] = __builtin_subc(u[j], v[j], br, &br);
        br = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) x1[j] = __builtin_subc(x1[j], x2[j], br, &br);
        if (br) {
            uint32_t c = 0;
#pragma unroll
            for (int j = 0; j < 8; j++) x1[j] = __builtin_addc(x1[j], FrP::P[j], c, &c);
        }
        strip(u, x1);  // the difference of two odd numbers is even (and not 0)
    }
    Fr r;
    const uint32_t *x = is_one(u) ? x1 : x2;
#pragma unroll
    for (int j = 0; j < 8; j++) r.v[j] = x[j];
    // the plain inverse of a R is a^-1 R^-1: times R^3 (= R2 R2 / R) gives a^-1 R
    return r * (Fr::r2() * Fr::r2());
}
// canonical compare a > b (gt_zkp, zk_function.cu:3-22)
template <class P>
PNP_HD bool gt(const Fp<P> &a, const Fp<P> &b) {
    for (int i = P::N - 1; i >= 0; i--) {
        if (a.v[i] > b.v[i]) return true;
        if (a.v[i] < b.v[i]) return false;
    }
    return false;
}

// ---- memory helpers: 32-byte Fr as two 16-byte accesses ----
__device__ __forceinline__ Fr load_fr(const uint64_t *base, uint64_t i) {
    const uint4 *p = reinterpret_cast<const uint4 *>(base + 4 * i);
    uint4 lo = p[0], hi = p[1];
    Fr r;
    r.v[0] = lo.x; r.v[1] = lo.y; r.v[2] = lo.z; r.v[3] = lo.w;
    r.v[4] = hi.x; r.v[5] = hi.y; r.v[6] = hi.z; r.v[7] = hi.w;
    return r;
}
__device__ __forceinline__ void store_fr(uint64_t *base, uint64_t i, const Fr &a) {
    uint4 *p = reinterpret_cast<uint4 *>(base + 4 * i);
    p[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
    p[1] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
}
__device__ __forceinline__ Fq load_fq(const uint64_t *base) {
    const uint4 *p = reinterpret_cast<const uint4 *>(base);
    uint4 a = p[0], b = p[1], c = p[2];
    Fq r;
    r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
    r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
    r.v[8] = c.x; r.v[9] = c.y; r.v[10] = c.z; r.v[11] = c.w;
    return r;
}
__device__ __forceinline__ void store_fq(uint64_t *base, const Fq &a) {
    uint4 *p = reinterpret_cast<uint4 *>(base);
    p[0] = make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
    p[1] = make_uint4(a.v[4], a.v[5], a.v[6], a.v[7]);
    p[2] = make_uint4(a.v[8], a.v[9], a.v[10], a.v[11]);
}

// host-side conversion helpers (u64 limbs <-> Fp)
template <class P>
inline Fp<P> from_u64_limbs(const uint64_t *l) {
    Fp<P> r;
    for (int i = 0; i < P::N / 2; i++) {
        r.v[2 * i] = (uint32_t)l[i];
        r.v[2 * i + 1] = (uint32_t)(l[i] >> 32);
    }
    return r;
}
template <class P>
inline void to_u64_limbs(const Fp<P> &a, uint64_t *l) {
    for (int i = 0; i < P::N / 2; i++) l[i] = (uint64_t)a.v[2 * i] | ((uint64_t)a.v[2 * i + 1] << 32);
}

}  // namespace pnp
