/*
 * oracle/synth.c — CPU mirror of the synthetic-instance generators of the
 * HIP library (zprize23-gpu-submission_amd/csrc/synth.hip, poly.hip
 * k_random_fr_), so a full-size (n = 2^22) instance that bench.py builds on
 * the GPU can be rebuilt here and proved by the CPU restatement.
 * TEST INFRASTRUCTURE ONLY (see pnp_oracle.h).
 *
 * These are not reference functions: they generate inputs (a satisfying
 * random arithmetic circuit of the Merkle circuit's shape, SURVEY 8(d)
 * config 4), and tests/test_gpu_prove.py checks GPU == CPU generation.
 */
#include "oracle_internal.h"

static inline uint64_t splitmix(uint64_t x) {
    x += 0x9e3779b97f4a7c15ULL;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
    return x ^ (x >> 31);
}

/* k_random_fr_: 4 splitmix words, top bit cleared, reduced once; the value is
 * used directly as a Montgomery residue */
void or_synth_random_fr(uint64_t *d, uint64_t n, uint64_t seed) {
#pragma omp parallel for schedule(static)
    for (int64_t ii = 0; ii < (int64_t)n; ii++) {
        uint64_t i = (uint64_t)ii, h = seed * 0x2545F4914F6CDD1DULL + i * 4, r[4];
        for (int k = 0; k < 4; k++) r[k] = splitmix(h + k);
        r[3] &= 0x7fffffffffffffffULL;
        if (!or_gt_n(OR_FR_P, r, 4)) {  /* r >= p: subtract once */
            unsigned __int128 br = 0;
            for (int k = 0; k < 4; k++) {
                unsigned __int128 t = (unsigned __int128)r[k] - OR_FR_P[k] - (uint64_t)br;
                r[k] = (uint64_t)t;
                br = (t >> 64) & 1;
            }
        }
        memcpy(d + 4 * i, r, 32);
    }
}

static uint64_t gcd64(uint64_t x, uint64_t y) {
    while (y) { uint64_t t = x % y; x = y; y = t; }
    return x;
}

/* k_synth_circuit (synth.hip): w[0] = a (in), w[1] = b, w[2] = c (out),
 * w[3] = d (in); sel[0..7] = q_l q_r q_o q_4 q_c q_hl q_hr q_h4 (in, n rows),
 * sel[8] = q_arith (out); sigma[0..3] out (n rows, Montgomery) */
void or_synth_circuit(uint64_t *const w[4], uint64_t *const sel[9], uint64_t *const sigma[4],
                      uint64_t n, uint64_t ng, uint64_t pi_pos, const uint64_t pi_canon[4]) {
    uint64_t A = 0x9E3779B1ULL % ng;
    if (ng <= 2) A = 1;
    while (gcd64(A, ng) != 1) A++;
    uint32_t lg = 0;
    while ((1ULL << lg) < n) lg++;
    uint64_t omega[4], k1[4], k2[4], k3[4], pi[4];
    or_root_of_unity(omega, lg);
    or_fr_from_u64(k1, 7);
    or_fr_from_u64(k2, 13);
    or_fr_from_u64(k3, 17);
    or_fr_to_mont(pi, pi_canon);
    /* sigma_0 is written at row pi(i) by row i: fill the identity part first */
    const int64_t CH = 1024;
#pragma omp parallel for schedule(static)
    for (int64_t c = 0; c < (int64_t)((n + CH - 1) / CH); c++) {
        uint64_t lo = (uint64_t)c * CH, hi = lo + CH < n ? lo + CH : n, wi[4];
        or_fr_pow(wi, omega, lo);
        for (uint64_t i = lo; i < hi; i++) {
            or_fr_mul(sigma[2] + 4 * i, k2, wi);
            or_fr_mul(sigma[3] + 4 * i, k3, wi);
            if (i >= ng) {
                fr_copy(sigma[0] + 4 * i, wi);
                or_fr_mul(sigma[1] + 4 * i, k1, wi);
                fr_zero(sel[8] + 4 * i);
            }
            or_fr_mul(wi, wi, omega);
        }
    }
#pragma omp parallel for schedule(static)
    for (int64_t c = 0; c < (int64_t)((ng + CH - 1) / CH); c++) {
        uint64_t lo = (uint64_t)c * CH, hi = lo + CH < ng ? lo + CH : ng, wi[4];
        or_fr_pow(wi, omega, lo);
        for (uint64_t i = lo; i < hi; i++) {
            uint64_t pii = (uint64_t)(((unsigned __int128)A * i + 1) % ng);
            const uint64_t *ai = w[0] + 4 * i, *bi = w[0] + 4 * pii, *di = w[3] + 4 * i;
            fr_copy(w[1] + 4 * i, bi);
            or_fr_pow(sigma[1] + 4 * i, omega, pii);
            or_fr_mul(sigma[0] + 4 * pii, k1, wi);
            uint64_t acc[4], t[4], p[4], x2[4];
            or_fr_mul(acc, sel[0] + 4 * i, ai);
            or_fr_mul(t, sel[1] + 4 * i, bi); or_fr_add(acc, acc, t);
            or_fr_mul(t, sel[3] + 4 * i, di); or_fr_add(acc, acc, t);
            const uint64_t *vv[3] = {ai, bi, di};
            for (int j = 0; j < 3; j++) {
                or_fr_mul(x2, vv[j], vv[j]);
                or_fr_mul(p, x2, x2);
                or_fr_mul(p, p, vv[j]);
                or_fr_mul(t, sel[5 + j] + 4 * i, p);
                or_fr_add(acc, acc, t);
            }
            or_fr_add(acc, acc, sel[4] + 4 * i);
            if (i == pi_pos) or_fr_add(acc, acc, pi);
            or_fr_neg(acc, acc);
            or_fr_inv(t, sel[2] + 4 * i);
            or_fr_mul(w[2] + 4 * i, acc, t);
            fr_copy(sel[8] + 4 * i, OR_FR_ONE);
            or_fr_mul(wi, wi, omega);
        }
    }
}

/* k_coset_consts: x_i = 7 w_8n^i, vh_i = x_i^n - 1 (either may be NULL) */
void or_synth_coset_consts(uint64_t *vh, uint64_t *x, uint32_t lg) {
    uint64_t n = 1ULL << lg, N8 = n << 3, w8n[4], w8[4], g[4], gn[4], h[8][4];
    or_root_of_unity(w8n, lg + 3);
    or_root_of_unity(w8, 3);
    or_fr_from_u64(g, 7);
    or_fr_pow(gn, g, n);
    uint64_t p[4];
    fr_copy(p, gn);
    for (int k = 0; k < 8; k++) {
        or_fr_sub(h[k], p, OR_FR_ONE);
        or_fr_mul(p, p, w8);
    }
    const int64_t CH = 4096;
#pragma omp parallel for schedule(static)
    for (int64_t c = 0; c < (int64_t)((N8 + CH - 1) / CH); c++) {
        uint64_t lo = (uint64_t)c * CH, hi = lo + CH < N8 ? lo + CH : N8, xi[4];
        or_fr_pow(xi, w8n, lo);
        or_fr_mul(xi, xi, g);
        for (uint64_t i = lo; i < hi; i++) {
            if (x) fr_copy(x + 4 * i, xi);
            if (vh) fr_copy(vh + 4 * i, h[i & 7]);
            or_fr_mul(xi, xi, w8n);
        }
    }
}
