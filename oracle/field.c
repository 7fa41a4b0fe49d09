/*
 * oracle/field.c — BLS12-381 Fr / Fq Montgomery arithmetic (CPU restatement).
 * TEST INFRASTRUCTURE ONLY (see pnp_oracle.h).
 *
 * Restates lib/PLONK/utils/mont/cuda/ff/mont_t.cuh (mul :396-416,
 * pow :446-468, inverse :1064-1132) with the constants of
 * lib/PLONK/utils/mont/cuda/ff/bls12-381.hpp:7-93 and PLONK/src/bls12_381/
 * {fr,fq}.cuh.  64-bit limbs, CIOS Montgomery multiplication, values always
 * fully reduced (the reference stores canonical Montgomery residues).
 * Inversion is Fermat a^(p-2), so inv(0) = 0 as in the reference kernels.
 */
#include "oracle_internal.h"

const uint64_t OR_FR_P[4] = {0xffffffff00000001ULL, 0x53bda402fffe5bfeULL,
                             0x3339d80809a1d805ULL, 0x73eda753299d7d48ULL};
const uint64_t OR_FR_ONE[4] = {0x00000001fffffffeULL, 0x5884b7fa00034802ULL,
                               0x998c4fefecbc4ff5ULL, 0x1824b159acc5056fULL};
const uint64_t OR_FR_R2[4] = {0xc999e990f3f29c6dULL, 0x2b6cedcb87925c23ULL,
                              0x05d314967254398fULL, 0x0748d9d99f59ff11ULL};
static const uint64_t FR_INV = 0xfffffffeffffffffULL;

const uint64_t OR_FQ_P[6] = {0xb9feffffffffaaabULL, 0x1eabfffeb153ffffULL,
                             0x6730d2a0f6b0f624ULL, 0x64774b84f38512bfULL,
                             0x4b1ba7b6434bacd7ULL, 0x1a0111ea397fe69aULL};
const uint64_t OR_FQ_ONE[6] = {0x760900000002fffdULL, 0xebf4000bc40c0002ULL,
                               0x5f48985753c758baULL, 0x77ce585370525745ULL,
                               0x5c071a97a256ec6dULL, 0x15f65ec3fa80e493ULL};
const uint64_t OR_FQ_R2[6] = {0xf4df1f341c341746ULL, 0x0a76e6a609d104f1ULL,
                              0x8de5476c4c95b6d5ULL, 0x67eb88a9939d83c0ULL,
                              0x9a793e85b519952dULL, 0x11988fe592cae3aaULL};
static const uint64_t FQ_INV = 0x89f3fffcfffcfffdULL;

/* fr.cuh:42 TWO_ADIC_ROOT_OF_UNITY (Montgomery), fr.cuh:50 GENERATOR = 7 */
const uint64_t OR_FR_ROOT32[4] = {13381757501831005802ULL, 6564924994866501612ULL,
                                  789602057691799140ULL, 6625830629041353339ULL};
const uint64_t OR_FR_GEN[4] = {64424509425ULL, 1721329240476523535ULL,
                               18418692815241631664ULL, 3824455624000121028ULL};

/* ---------------- generic N-limb helpers ---------------- */
static inline int geq_n(const uint64_t *a, const uint64_t *p, int N) {
    for (int i = N - 1; i >= 0; i--) {
        if (a[i] > p[i]) return 1;
        if (a[i] < p[i]) return 0;
    }
    return 1;
}
static inline uint64_t sub_n(uint64_t *r, const uint64_t *a, const uint64_t *b, int N) {
    uint64_t borrow = 0;
    for (int i = 0; i < N; i++) {
        u128 d = (u128)a[i] - b[i] - borrow;
        r[i] = (uint64_t)d;
        borrow = (uint64_t)(d >> 64) & 1;
    }
    return borrow;
}
static inline uint64_t add_n(uint64_t *r, const uint64_t *a, const uint64_t *b, int N) {
    uint64_t c = 0;
    for (int i = 0; i < N; i++) {
        u128 s = (u128)a[i] + b[i] + c;
        r[i] = (uint64_t)s;
        c = (uint64_t)(s >> 64);
    }
    return c;
}
static inline void addmod_n(uint64_t *r, const uint64_t *a, const uint64_t *b,
                            const uint64_t *p, int N) {
    uint64_t t[6];
    uint64_t c = add_n(t, a, b, N);
    if (c || geq_n(t, p, N)) sub_n(t, t, p, N);
    for (int i = 0; i < N; i++) r[i] = t[i];
}
static inline void submod_n(uint64_t *r, const uint64_t *a, const uint64_t *b,
                            const uint64_t *p, int N) {
    uint64_t t[6];
    uint64_t bw = sub_n(t, a, b, N);
    if (bw) add_n(t, t, p, N);
    for (int i = 0; i < N; i++) r[i] = t[i];
}
/* CIOS Montgomery multiplication (mont_t.cuh:396-416 restated on 64-bit limbs) */
static inline void mont_mul_n(uint64_t *r, const uint64_t *a, const uint64_t *b,
                              const uint64_t *p, uint64_t inv, int N) {
    uint64_t t[8] = {0};
    for (int i = 0; i < N; i++) {
        uint64_t c = 0;
        for (int j = 0; j < N; j++) {
            u128 s = (u128)a[j] * b[i] + t[j] + c;
            t[j] = (uint64_t)s;
            c = (uint64_t)(s >> 64);
        }
        u128 s = (u128)t[N] + c;
        t[N] = (uint64_t)s;
        t[N + 1] = (uint64_t)(s >> 64);
        uint64_t m = t[0] * inv;
        s = (u128)m * p[0] + t[0];
        c = (uint64_t)(s >> 64);
        for (int j = 1; j < N; j++) {
            s = (u128)m * p[j] + t[j] + c;
            t[j - 1] = (uint64_t)s;
            c = (uint64_t)(s >> 64);
        }
        s = (u128)t[N] + c;
        t[N - 1] = (uint64_t)s;
        t[N] = t[N + 1] + (uint64_t)(s >> 64);
    }
    if (t[N] || geq_n(t, p, N)) sub_n(t, t, p, N);
    for (int i = 0; i < N; i++) r[i] = t[i];
}

/* ---------------- Fr ---------------- */
void or_fr_add(uint64_t r[4], const uint64_t a[4], const uint64_t b[4]) { addmod_n(r, a, b, OR_FR_P, 4); }
void or_fr_sub(uint64_t r[4], const uint64_t a[4], const uint64_t b[4]) { submod_n(r, a, b, OR_FR_P, 4); }
void or_fr_mul(uint64_t r[4], const uint64_t a[4], const uint64_t b[4]) { mont_mul_n(r, a, b, OR_FR_P, FR_INV, 4); }
void or_fr_neg(uint64_t r[4], const uint64_t a[4]) {
    static const uint64_t z[4] = {0, 0, 0, 0};
    submod_n(r, z, a, OR_FR_P, 4);
}
void or_fr_to_mont(uint64_t r[4], const uint64_t a[4]) { or_fr_mul(r, a, OR_FR_R2); }
void or_fr_from_mont(uint64_t r[4], const uint64_t a[4]) {
    static const uint64_t one[4] = {1, 0, 0, 0};
    or_fr_mul(r, a, one);
}
/* exp_mod (mont_arithmetic.cu:89 exp_mod_kernel_) with a u64 exponent */
void or_fr_pow(uint64_t r[4], const uint64_t a[4], uint64_t e) {
    uint64_t acc[4], base[4];
    fr_copy(acc, OR_FR_ONE);
    fr_copy(base, a);
    while (e) {
        if (e & 1) or_fr_mul(acc, acc, base);
        or_fr_mul(base, base, base);
        e >>= 1;
    }
    fr_copy(r, acc);
}
static void pow_big(uint64_t *r, const uint64_t *a, const uint64_t *e, int N,
                    const uint64_t *one, void (*mul)(uint64_t *, const uint64_t *, const uint64_t *)) {
    uint64_t acc[6], base[6];
    for (int i = 0; i < N; i++) { acc[i] = one[i]; base[i] = a[i]; }
    for (int w = 0; w < N; w++)
        for (int b = 0; b < 64; b++) {
            if ((e[w] >> b) & 1) mul(acc, acc, base);
            mul(base, base, base);
        }
    for (int i = 0; i < N; i++) r[i] = acc[i];
}
static void fr_mul_v(uint64_t *r, const uint64_t *a, const uint64_t *b) { or_fr_mul(r, a, b); }
static void fq_mul_v(uint64_t *r, const uint64_t *a, const uint64_t *b) { or_fq_mul(r, a, b); }
/* inv_mod (mont_arithmetic.cu:73 inv_mod_kernel_): a^(p-2) */
void or_fr_inv(uint64_t r[4], const uint64_t a[4]) {
    uint64_t e[4];
    static const uint64_t two[4] = {2, 0, 0, 0};
    sub_n(e, OR_FR_P, two, 4);
    pow_big(r, a, e, 4, OR_FR_ONE, fr_mul_v);
}
int or_fr_is_zero(const uint64_t a[4]) { return (a[0] | a[1] | a[2] | a[3]) == 0; }
int or_fr_eq(const uint64_t a[4], const uint64_t b[4]) {
    return a[0] == b[0] && a[1] == b[1] && a[2] == b[2] && a[3] == b[3];
}
/* fr::make_tensor(x) (fr.cuh:57-64): small integer into Montgomery form */
void or_fr_from_u64(uint64_t r[4], uint64_t x) {
    uint64_t t[4] = {x, 0, 0, 0};
    or_fr_to_mont(r, t);
}

/* ---------------- Fq ---------------- */
void or_fq_add(uint64_t r[6], const uint64_t a[6], const uint64_t b[6]) { addmod_n(r, a, b, OR_FQ_P, 6); }
void or_fq_sub(uint64_t r[6], const uint64_t a[6], const uint64_t b[6]) { submod_n(r, a, b, OR_FQ_P, 6); }
void or_fq_mul(uint64_t r[6], const uint64_t a[6], const uint64_t b[6]) { mont_mul_n(r, a, b, OR_FQ_P, FQ_INV, 6); }
void or_fq_neg(uint64_t r[6], const uint64_t a[6]) {
    static const uint64_t z[6] = {0};
    submod_n(r, z, a, OR_FQ_P, 6);
}
void or_fq_to_mont(uint64_t r[6], const uint64_t a[6]) { or_fq_mul(r, a, OR_FQ_R2); }
void or_fq_from_mont(uint64_t r[6], const uint64_t a[6]) {
    static const uint64_t one[6] = {1, 0, 0, 0, 0, 0};
    or_fq_mul(r, a, one);
}
void or_fq_inv(uint64_t r[6], const uint64_t a[6]) {
    uint64_t e[6];
    static const uint64_t two[6] = {2, 0, 0, 0, 0, 0};
    sub_n(e, OR_FQ_P, two, 6);
    pow_big(r, a, e, 6, OR_FQ_ONE, fq_mul_v);
}
int or_fq_is_zero(const uint64_t a[6]) {
    return (a[0] | a[1] | a[2] | a[3] | a[4] | a[5]) == 0;
}
int or_fq_eq(const uint64_t a[6], const uint64_t b[6]) {
    for (int i = 0; i < 6; i++)
        if (a[i] != b[i]) return 0;
    return 1;
}
/* gt_zkp (zk_function.cu:3-22): lexicographic compare from the top limb */
int or_gt_n(const uint64_t *a, const uint64_t *b, int N) {
    for (int i = N - 1; i >= 0; i--) {
        if (a[i] > b[i]) return 1;
        if (a[i] < b[i]) return 0;
    }
    return 0;
}

/* ---------------- vectors ---------------- */
void or_fr_vec_to_mont(uint64_t *v, uint64_t n) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)n; i++) or_fr_to_mont(v + 4 * i, v + 4 * i);
}
void or_fr_vec_from_mont(uint64_t *v, uint64_t n) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)n; i++) or_fr_from_mont(v + 4 * i, v + 4 * i);
}

int or_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* the CPU baseline runs on every core the process may use,
   whatever OMP_NUM_THREADS the environment inherited */
void or_set_num_threads(int t) {
#ifdef _OPENMP
    if (t > 0) omp_set_num_threads(t);
#else
    (void)t;
#endif
}
