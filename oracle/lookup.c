/*
 * oracle/lookup.c — plookup pieces of the CPU prover (ZK-Garage plonk-core,
 * prover.rs:304-307 and permutation/mod.rs:754-822).
 * TEST INFRASTRUCTURE ONLY (see pnp_oracle.h).
 *
 *   or_combine_split  MultiSet::combine_split (lookup/multiset.rs:131-180):
 *                     the values of t and f grouped by value, groups in the
 *                     order of first occurrence in t, each group's copies
 *                     split between the even half h1 and the odd half h2
 *                     (an odd group alternates starting with h1).  Every f
 *                     value must occur in t (Error::ElementNotIndexed).
 *   or_lookup_z2      compute_lookup_permutation_poly with t_next[i] =
 *                     t[i + 1], h1_next[i] = h1[i + 1] (wrapping), coefficients.
 */
#include "oracle_internal.h"

typedef struct {
    uint64_t v[4];
    uint64_t tag; /* < n: position in t; >= n: n + position in f */
} rec_t;

static int rec_cmp(const void *pa, const void *pb) {
    const rec_t *a = (const rec_t *)pa, *b = (const rec_t *)pb;
    for (int k = 3; k >= 0; k--) {
        if (a->v[k] != b->v[k]) return a->v[k] < b->v[k] ? -1 : 1;
    }
    return a->tag < b->tag ? -1 : a->tag > b->tag;
}

typedef struct {
    uint64_t first, start, len;
} run_t;

static int run_cmp(const void *pa, const void *pb) {
    const run_t *a = (const run_t *)pa, *b = (const run_t *)pb;
    return a->first < b->first ? -1 : a->first > b->first;
}

int or_combine_split(const uint64_t *t, const uint64_t *f, uint64_t n, uint64_t *h1, uint64_t *h2) {
    rec_t *r = (rec_t *)malloc(sizeof(rec_t) * 2 * n);
    for (uint64_t i = 0; i < n; i++) {
        memcpy(r[i].v, t + 4 * i, 32);
        r[i].tag = i;
        memcpy(r[n + i].v, f + 4 * i, 32);
        r[n + i].tag = n + i;
    }
    qsort(r, 2 * n, sizeof(rec_t), rec_cmp);
    run_t *runs = (run_t *)malloc(sizeof(run_t) * 2 * n);
    uint64_t nr = 0;
    for (uint64_t i = 0; i < 2 * n; i++) {
        if (i == 0 || memcmp(r[i].v, r[i - 1].v, 32) != 0) {
            if (r[i].tag >= n) { /* an f value absent from t */
                free(r);
                free(runs);
                return PNP_E_ARG;
            }
            runs[nr].first = r[i].tag;
            runs[nr].start = i;
            runs[nr].len = 0;
            nr++;
        }
        runs[nr - 1].len++;
    }
    qsort(runs, nr, sizeof(run_t), run_cmp);
    uint64_t e = 0, o = 0;
    int parity = 0;
    for (uint64_t k = 0; k < nr; k++) {
        const uint64_t *v = r[runs[k].start].v;
        uint64_t c = runs[k].len, half = c / 2;
        for (uint64_t j = 0; j < half; j++) {
            memcpy(h1 + 4 * e++, v, 32);
            memcpy(h2 + 4 * o++, v, 32);
        }
        if (c & 1) {
            if (parity) memcpy(h2 + 4 * o++, v, 32);
            else memcpy(h1 + 4 * e++, v, 32);
            parity ^= 1;
        }
    }
    free(r);
    free(runs);
    return (e == n && o == n) ? PNP_OK : PNP_E_ARG;
}

uint64_t *or_lookup_z2(uint32_t lg, const uint64_t *f, const uint64_t *t, const uint64_t *h1,
                       const uint64_t *h2, const uint64_t delta[4], const uint64_t eps[4]) {
    uint64_t n = 1ULL << lg;
    uint64_t opd[4], eopd[4];
    or_fr_add(opd, delta, OR_FR_ONE);
    or_fr_mul(eopd, eps, opd);
    uint64_t *num = (uint64_t *)calloc(n, 32), *den = (uint64_t *)calloc(n, 32);
#pragma omp parallel for schedule(static)
    for (int64_t ii = 0; ii < (int64_t)n; ii++) {
        uint64_t i = (uint64_t)ii, nx = (i + 1) & (n - 1);
        uint64_t a[4], b[4], c[4], d[4], x[4];
        /* (1+delta)(eps + f)(eps(1+delta) + t + delta t_next) */
        or_fr_add(a, eps, f + 4 * i);
        or_fr_mul(a, opd, a);
        or_fr_add(b, eopd, t + 4 * i);
        or_fr_mul(x, delta, t + 4 * nx);
        or_fr_add(b, b, x);
        or_fr_mul(a, a, b);
        /* (eps(1+delta) + h1 + delta h2)(eps(1+delta) + h2 + delta h1_next) */
        or_fr_add(c, eopd, h1 + 4 * i);
        or_fr_mul(x, h2 + 4 * i, delta);
        or_fr_add(c, c, x);
        or_fr_add(d, eopd, h2 + 4 * i);
        or_fr_mul(x, h1 + 4 * nx, delta);
        or_fr_add(d, d, x);
        or_fr_mul(c, c, d);
        memcpy(num + 4 * i, a, 32);
        memcpy(den + 4 * i, c, 32);
    }
    or_batch_inverse(den, n);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)n; i++) or_fr_mul(num + 4 * i, num + 4 * i, den + 4 * i);
    /* p_0 = 1, p_i = prod_{k < i} ratio_k */
    or_prefix_product(num, n);
    or_ntt(num, lg, 1, 0);
    free(den);
    return num;
}
