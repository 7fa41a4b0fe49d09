/*
 * oracle/poly.c — radix-2 NTT (arkworks Radix2EvaluationDomain semantics) and
 * polynomial helpers.  TEST INFRASTRUCTURE ONLY (see pnp_oracle.h).
 *
 * Reference semantics restated:
 *   domain / roots      : PLONK/src/domain.cu:12-36 (omega_k = ROOT32^(2^(32-k)))
 *   Ntt / Intt          : utils/function.cu:249-259 -> zksnark_ntt.cu:74-92 ->
 *                         ntt_kernel/ntt.cuh:57-144 (natural order in and out,
 *                         inverse multiplies by n^-1)
 *   Ntt_coset/Intt_coset: function.cu:261-273, kernels.cuh:116-140
 *                         (forward: x_i *= g^i first; inverse: x_i *= g^-i last;
 *                         g = 7, parameters/bls12_381.h group_gen)
 *   evaluate            : function.cu:162-173 (sum c_i x^i)
 *   poly_div_poly       : mont_arithmetic.cu:305-331 (quotient by X - z)
 *   accumulate_mul_poly : mont_arithmetic.cu:334-360 (exclusive prefix product)
 */
#include "oracle_internal.h"

void or_root_of_unity(uint64_t r[4], uint32_t lg) {
    /* get_root_of_unity (domain.cu:29-36) */
    or_fr_pow(r, OR_FR_ROOT32, 1ULL << (32 - lg));
}

static uint64_t bitrev(uint64_t x, uint32_t lg) {
    uint64_t r = 0;
    for (uint32_t i = 0; i < lg; i++) { r = (r << 1) | (x & 1); x >>= 1; }
    return r;
}

static void ntt_core(uint64_t *v, uint32_t lg_n, const uint64_t root[4]) {
    uint64_t n = 1ULL << lg_n;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t j = bitrev(i, lg_n);
        if (i < j) {
            uint64_t t[4];
            fr_copy(t, v + 4 * i);
            fr_copy(v + 4 * i, v + 4 * j);
            fr_copy(v + 4 * j, t);
        }
    }
    uint64_t *tw = (uint64_t *)malloc(sizeof(uint64_t) * 4 * (n / 2 + 1));
    for (uint32_t s = 1; s <= lg_n; s++) {
        uint64_t m = 1ULL << s, half = m >> 1;
        uint64_t wm[4];
        or_fr_pow(wm, root, n / m);
        fr_copy(tw, OR_FR_ONE);
        for (uint64_t j = 1; j < half; j++) or_fr_mul(tw + 4 * j, tw + 4 * (j - 1), wm);
#pragma omp parallel for schedule(static) if (n >= 4096)
        for (int64_t idx = 0; idx < (int64_t)(n / 2); idx++) {
            uint64_t k = ((uint64_t)idx / half) * m, j = (uint64_t)idx % half;
            uint64_t *a = v + 4 * (k + j), *b = v + 4 * (k + j + half);
            uint64_t t[4];
            or_fr_mul(t, b, tw + 4 * j);
            or_fr_sub(b, a, t);
            or_fr_add(a, a, t);
        }
    }
    free(tw);
}

static void distribute_powers(uint64_t *v, uint64_t n, const uint64_t g[4]) {
    /* x_i *= g^i (LDE_distribute_powers, kernels.cuh:116-140) */
    const int64_t CH = 1024;
#pragma omp parallel for schedule(static)
    for (int64_t c = 0; c < (int64_t)((n + CH - 1) / CH); c++) {
        uint64_t start = (uint64_t)c * CH, end = start + CH < n ? start + CH : n;
        uint64_t p[4];
        or_fr_pow(p, g, start);
        for (uint64_t i = start; i < end; i++) {
            or_fr_mul(v + 4 * i, v + 4 * i, p);
            or_fr_mul(p, p, g);
        }
    }
}

void or_ntt(uint64_t *v, uint32_t lg_n, int inverse, int coset) {
    uint64_t n = 1ULL << lg_n;
    uint64_t root[4];
    or_root_of_unity(root, lg_n);
    if (!inverse) {
        if (coset) distribute_powers(v, n, OR_FR_GEN);
        ntt_core(v, lg_n, root);
    } else {
        uint64_t rinv[4], ninv[4], nf[4];
        or_fr_inv(rinv, root);
        ntt_core(v, lg_n, rinv);
        or_fr_from_u64(nf, n);
        or_fr_inv(ninv, nf);
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < (int64_t)n; i++) or_fr_mul(v + 4 * i, v + 4 * i, ninv);
        if (coset) {
            uint64_t ginv[4];
            or_fr_inv(ginv, OR_FR_GEN);
            distribute_powers(v, n, ginv);
        }
    }
}

void or_coset_lde8(const uint64_t *coeffs, uint64_t *out8, uint32_t lg_n) {
    /* Ntt_coset::forward (function.cu:264-267): pad_poly to 8n then coset NTT */
    uint64_t n = 1ULL << lg_n;
    memcpy(out8, coeffs, 32 * n);
    memset(out8 + 4 * n, 0, 32 * 7 * n);
    or_ntt(out8, lg_n + 3, 0, 1);
}

void or_poly_eval(const uint64_t *c, uint64_t n, const uint64_t x[4], uint64_t out[4]) {
    uint64_t acc[4] = {0, 0, 0, 0};
    for (int64_t i = (int64_t)n - 1; i >= 0; i--) {
        or_fr_mul(acc, acc, x);
        or_fr_add(acc, acc, c + 4 * i);
    }
    fr_copy(out, acc);
}

void or_poly_div_linear(uint64_t *p, uint64_t n, const uint64_t z[4]) {
    /* q_k = sum_{j>k} p_j z^(j-k-1), q_{n-1} = 0 */
    uint64_t acc[4] = {0, 0, 0, 0};
    for (int64_t k = (int64_t)n - 1; k >= 0; k--) {
        uint64_t pk[4];
        fr_copy(pk, p + 4 * k);
        fr_copy(p + 4 * k, acc);
        or_fr_mul(acc, acc, z);
        or_fr_add(acc, acc, pk);
    }
}

void or_prefix_product(uint64_t *v, uint64_t n) {
    uint64_t acc[4];
    fr_copy(acc, OR_FR_ONE);
    for (uint64_t i = 0; i < n; i++) {
        uint64_t t[4];
        fr_copy(t, v + 4 * i);
        fr_copy(v + 4 * i, acc);
        or_fr_mul(acc, acc, t);
    }
}

void or_batch_inverse(uint64_t *v, uint64_t n) {
    /* per-element inverse (inv_mod_kernel_, mont_arithmetic.cu:73), computed
     * with Montgomery's trick over chunks; zeros map to zero. */
    const int64_t CH = 256;
#pragma omp parallel for schedule(static)
    for (int64_t c = 0; c < (int64_t)((n + CH - 1) / CH); c++) {
        uint64_t start = (uint64_t)c * CH, end = start + CH < n ? start + CH : n;
        uint64_t pre[256][4], acc[4], inv[4];
        fr_copy(acc, OR_FR_ONE);
        for (uint64_t i = start; i < end; i++) {
            fr_copy(pre[i - start], acc);
            if (!or_fr_is_zero(v + 4 * i)) or_fr_mul(acc, acc, v + 4 * i);
        }
        or_fr_inv(inv, acc);
        for (int64_t i = (int64_t)end - 1; i >= (int64_t)start; i--) {
            if (or_fr_is_zero(v + 4 * i)) continue;
            uint64_t t[4];
            or_fr_mul(t, inv, pre[i - start]);
            or_fr_mul(inv, inv, v + 4 * i);
            fr_copy(v + 4 * i, t);
        }
    }
}
