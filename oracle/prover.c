/*
 * oracle/prover.c — CPU restatement of gen_proof.
 * TEST INFRASTRUCTURE ONLY (see pnp_oracle.h).
 *
 * Semantics: the ZK-Garage CPU prover Prover::prove_with_preprocessed
 * (plonk-core/src/proof_system/prover.rs:171-660, quotient_poly.rs,
 * linearisation_poly.rs, the widget sources, permutation/mod.rs:629-822), which the
 * north star names as the parity target, in the protocol order of the GPU
 * path it replaces (lib/PLONK/src/gen_proof.cuh:10-489).  On the reference's
 * own circuit class (the Merkle circuit: no custom gates, no lookup tables,
 * one public input) the two reference paths coincide, and so does this
 * restatement.  Outside it the GPU path takes shortcuts that make its proofs
 * fail verification (combine_split skipped, q_m / custom-
 * selector / q_lookup coefficients treated as empty, the 8-byte t_next /
 * h1_next shift, "delta + h1_next" in the linearisation); this restatement
 * follows prover.rs there:
 *   - h1, h2 from combine_split (lookup.c);
 *   - z2 with t_next[i] = t[i+1], h1_next[i] = h1[i+1];
 *   - custom-gate widgets in the quotient AND the linearisation; q_m and
 *     q_lookup coefficients read whenever their evaluations are non-zero;
 *   - any number of public inputs (BTreeMap order, zeros dropped).
 * The transcript label is the caller's ("Merkle tree" for the v1 symbol,
 * gen_proof.cuh:19-22).
 */
#include "oracle_internal.h"
#include <stdio.h>

#define E4(p, i) ((p) + 4 * (uint64_t)(i))

static uint64_t *vec_alloc(uint64_t n) { return (uint64_t *)calloc(n ? n : 1, 32); }

static uint64_t next_pow2(uint64_t x) {
    uint64_t r = 1;
    while (r < x) r <<= 1;
    return r;
}
static uint32_t lg2(uint64_t x) {
    uint32_t l = 0;
    while ((1ULL << l) < x) l++;
    return l;
}

/* pad_poly (function.cu:203-210): copy m elements, zero to n */
static uint64_t *pad(const uint64_t *src, uint64_t m, uint64_t n) {
    uint64_t *v = vec_alloc(n);
    if (m > n) m = n;
    if (src && m) memcpy(v, src, 32 * m);
    return v;
}
static uint64_t *intt_copy(const uint64_t *evals, uint32_t lg) {
    uint64_t n = 1ULL << lg;
    uint64_t *v = vec_alloc(n);
    memcpy(v, evals, 32 * n);
    or_ntt(v, lg, 1, 0);
    return v;
}
static uint64_t *lde8(const uint64_t *coeffs, uint32_t lg) {
    uint64_t *v = vec_alloc(8ULL << lg);
    or_coset_lde8(coeffs, v, lg);
    return v;
}
static void commit_aff(const CommitKeyC *ck, const uint64_t *poly, uint64_t n, CommitmentC *out) {
    uint64_t aff[12];
    or_commit(ck->powers_of_g, poly, n, aff);
    memcpy(out->x, aff, 48);
    memcpy(out->y, aff + 48 / 8, 48);
}
static void append_comm(or_transcript *t, const char *label, const CommitmentC *c) {
    uint64_t aff[12];
    memcpy(aff, c->x, 48);
    memcpy(aff + 6, c->y, 48);
    or_transcript_append_point(t, label, aff);
}
static int all_zero(const uint64_t *v, uint64_t n) {
    for (uint64_t i = 0; i < 4 * n; i++)
        if (v[i]) return 0;
    return 1;
}

/* compress (zksnark_compute_query_table.cu:110-129): t0 + z t1 + z^2 t2 + z^3 t3 */
static void compress4(uint64_t *out, const uint64_t *t0, const uint64_t *t1,
                      const uint64_t *t2, const uint64_t *t3, const uint64_t z[4], uint64_t n) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)n; i++) {
        uint64_t acc[4];
        fr_copy(acc, E4(t3, i));
        or_fr_mul(acc, acc, z); or_fr_add(acc, acc, E4(t2, i));
        or_fr_mul(acc, acc, z); or_fr_add(acc, acc, E4(t1, i));
        or_fr_mul(acc, acc, z); or_fr_add(acc, acc, E4(t0, i));
        fr_copy(E4(out, i), acc);
    }
}

/* compute_permutation_poly (permutation/mod.cu:44-109) */
static uint64_t *permutation_poly(uint32_t lg, uint64_t *const w[4], const uint64_t beta[4],
                                  const uint64_t gamma[4], uint64_t *const sigma_coeffs[4]) {
    uint64_t n = 1ULL << lg;
    uint64_t *sig[4];
    for (int j = 0; j < 4; j++) {
        sig[j] = vec_alloc(n);
        memcpy(sig[j], sigma_coeffs[j], 32 * n);
        or_ntt(sig[j], lg, 0, 0);  /* NTT.forward(sigma_polys[j]) */
    }
    uint64_t ks[4][4], bk[4][4], omega[4];
    fr_copy(ks[0], OR_FR_ONE);
    or_fr_from_u64(ks[1], 7);   /* K1 (constants.cu:3-7) */
    or_fr_from_u64(ks[2], 13);  /* K2 */
    or_fr_from_u64(ks[3], 17);  /* K3 */
    for (int j = 0; j < 4; j++) or_fr_mul(bk[j], beta, ks[j]);
    or_root_of_unity(omega, lg);
    uint64_t *num = vec_alloc(n), *den = vec_alloc(n);
    const int64_t CH = 1024;
#pragma omp parallel for schedule(static)
    for (int64_t c = 0; c < (int64_t)((n + CH - 1) / CH); c++) {
        uint64_t start = (uint64_t)c * CH, end = start + CH < n ? start + CH : n;
        uint64_t root[4];
        or_fr_pow(root, omega, start);  /* gen_sequence: roots[i] = omega^i */
        for (uint64_t i = start; i < end; i++) {
            uint64_t nm[4], dn[4], t[4];
            fr_copy(nm, OR_FR_ONE);
            fr_copy(dn, OR_FR_ONE);
            for (int j = 0; j < 4; j++) {
                /* _numerator_irreducible: w + (beta*k)*root + gamma */
                or_fr_mul(t, bk[j], root);
                or_fr_add(t, E4(w[j], i), t);
                or_fr_add(t, t, gamma);
                or_fr_mul(nm, nm, t);
                /* _denominator_irreducible: w + sigma*beta + gamma */
                or_fr_mul(t, E4(sig[j], i), beta);
                or_fr_add(t, E4(w[j], i), t);
                or_fr_add(t, t, gamma);
                or_fr_mul(dn, dn, t);
            }
            fr_copy(E4(num, i), nm);
            fr_copy(E4(den, i), dn);
            or_fr_mul(root, root, omega);
        }
    }
    or_batch_inverse(den, n);  /* div_mod(extend_one, denominator_product) */
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)n; i++) or_fr_mul(E4(num, i), E4(num, i), E4(den, i));
    or_prefix_product(num, n);  /* accumulate_mul_poly */
    or_ntt(num, lg, 1, 0);
    for (int j = 0; j < 4; j++) free(sig[j]);
    free(den);
    return num;
}

static void fr_pow5(uint64_t r[4], const uint64_t a[4]) {
    uint64_t a2[4], a4[4];
    or_fr_mul(a2, a, a);
    or_fr_mul(a4, a2, a2);
    or_fr_mul(r, a4, a);
}

typedef struct {
    uint64_t alpha[4], beta[4], gamma[4], delta[4], eps[4], zeta[4];
    uint64_t range[4], logic[4], fixed[4], var[4], lsep[4];
} challenges_t;

/* selectors whose 8n evaluations are non-zero (the others are the zero
 * polynomial: their Rust coefficient Vecs are empty and never read) */
typedef struct {
    int q_m, range, logic, fixed, var, q_lookup;
} nz_t;

/* compute_quotient_poly (proof_system/quotient.cu:142-376) */
static uint64_t *quotient_poly(uint32_t lg, const ProverKeyC *pk, const challenges_t *ch, const nz_t *nz,
                               const uint64_t *z_poly, const uint64_t *z2_poly,
                               uint64_t *const wpoly[4], const uint64_t *pi_poly,
                               const uint64_t *f_poly, const uint64_t *table_poly,
                               const uint64_t *h1_poly, const uint64_t *h2_poly) {
    uint64_t n = 1ULL << lg, N8 = 8 * n;
    uint64_t *w8[4];
    for (int j = 0; j < 4; j++) w8[j] = lde8(wpoly[j], lg);
    uint64_t *z8 = lde8(z_poly, lg), *pi8 = lde8(pi_poly, lg);
    uint64_t *f8 = lde8(f_poly, lg), *t8 = lde8(table_poly, lg);
    uint64_t *h18 = lde8(h1_poly, lg), *h28 = lde8(h2_poly, lg), *z28 = lde8(z2_poly, lg);
    /* compute_first_lagrange_poly_scaled (quotient.cu:3-8) for alpha^2 and 1 */
    uint64_t alpha2[4];
    or_fr_mul(alpha2, ch->alpha, ch->alpha);
    uint64_t *l1a = vec_alloc(n), *l1 = vec_alloc(n);
    fr_copy(l1a, alpha2);
    fr_copy(l1, OR_FR_ONE);
    or_ntt(l1a, lg, 1, 0);
    or_ntt(l1, lg, 1, 0);
    uint64_t *l1a8 = lde8(l1a, lg), *l18 = lde8(l1, lg);
    uint64_t bk[4][4], ks[4][4];
    fr_copy(ks[0], OR_FR_ONE);
    or_fr_from_u64(ks[1], 7);
    or_fr_from_u64(ks[2], 13);
    or_fr_from_u64(ks[3], 17);
    for (int j = 0; j < 4; j++) or_fr_mul(bk[j], ch->beta, ks[j]);
    uint64_t opd[4], eopd[4], sep2[4], sep3[4];
    or_fr_add(opd, ch->delta, OR_FR_ONE);
    or_fr_mul(eopd, ch->eps, opd);
    or_fr_mul(sep2, ch->lsep, ch->lsep);
    or_fr_mul(sep3, sep2, ch->lsep);
    const uint64_t *sig8[4] = {pk->left_sigma_evals, pk->right_sigma_evals,
                               pk->out_sigma_evals, pk->fourth_sigma_evals};
    uint64_t *num = vec_alloc(N8);
#pragma omp parallel for schedule(static)
    for (int64_t ii = 0; ii < (int64_t)N8; ii++) {
        uint64_t i = (uint64_t)ii, nx = (i + 8) % N8;
        const uint64_t *a = E4(w8[0], i), *b = E4(w8[1], i), *c = E4(w8[2], i), *d = E4(w8[3], i);
        uint64_t t[4], acc[4], g[4];
        /* compute_quotient_i (widget/arithmetic.cu:7-45) */
        or_fr_mul(acc, a, b);
        or_fr_mul(acc, acc, E4(pk->q_m_evals, i));
        or_fr_mul(t, a, E4(pk->q_l_evals, i)); or_fr_add(acc, acc, t);
        or_fr_mul(t, b, E4(pk->q_r_evals, i)); or_fr_add(acc, acc, t);
        or_fr_mul(t, c, E4(pk->q_o_evals, i)); or_fr_add(acc, acc, t);
        or_fr_mul(t, d, E4(pk->q_4_evals, i)); or_fr_add(acc, acc, t);
        fr_pow5(t, a); or_fr_mul(t, t, E4(pk->q_hl_evals, i)); or_fr_add(acc, acc, t);
        fr_pow5(t, b); or_fr_mul(t, t, E4(pk->q_hr_evals, i)); or_fr_add(acc, acc, t);
        fr_pow5(t, d); or_fr_mul(t, t, E4(pk->q_h4_evals, i)); or_fr_add(acc, acc, t);
        or_fr_add(acc, acc, E4(pk->q_c_evals, i));
        or_fr_mul(g, acc, E4(pk->q_arith_evals, i));
        or_fr_add(g, g, E4(pi8, i));  /* + pi_eval_8n (quotient_poly.rs:240) */
        /* custom gates (quotient_poly.rs:253-296): selector * constraints */
        if (nz->range || nz->logic || nz->fixed || nz->var) {
            widget_vals wv = {a, b, c, d, E4(w8[0], nx), E4(w8[1], nx), E4(w8[3], nx),
                              E4(pk->q_l_evals, i), E4(pk->q_r_evals, i), E4(pk->q_c_evals, i)};
            if (nz->range) {
                or_w_range(t, ch->range, &wv);
                or_fr_mul(t, t, E4(pk->range_selector_evals, i));
                or_fr_add(g, g, t);
            }
            if (nz->logic) {
                or_w_logic(t, ch->logic, &wv);
                or_fr_mul(t, t, E4(pk->logic_selector_evals, i));
                or_fr_add(g, g, t);
            }
            if (nz->fixed) {
                or_w_fbsm(t, ch->fixed, &wv);
                or_fr_mul(t, t, E4(pk->fixed_group_add_selector_evals, i));
                or_fr_add(g, g, t);
            }
            if (nz->var) {
                or_w_cadd(t, ch->var, &wv);
                or_fr_mul(t, t, E4(pk->variable_group_add_selector_evals, i));
                or_fr_add(g, g, t);
            }
        }
        /* permutation_compute_quotient (proof_system/permutation.cu:267-296) */
        const uint64_t *x = E4(pk->linear_evaluations, i);
        uint64_t pa[4], pb[4], pc[4];
        fr_copy(pa, OR_FR_ONE);
        fr_copy(pb, OR_FR_ONE);
        const uint64_t *w4[4] = {a, b, c, d};
        for (int j = 0; j < 4; j++) {
            or_fr_mul(t, x, bk[j]);  /* x*beta (j=0) or x*(beta*k_j) */
            or_fr_add(t, t, w4[j]);
            or_fr_add(t, t, ch->gamma);
            or_fr_mul(pa, pa, t);
            or_fr_mul(t, E4(sig8[j], i), ch->beta);
            or_fr_add(t, t, w4[j]);
            or_fr_add(t, t, ch->gamma);
            or_fr_mul(pb, pb, t);
        }
        or_fr_mul(pa, pa, E4(z8, i));
        or_fr_mul(pa, pa, ch->alpha);
        or_fr_mul(pb, pb, E4(z8, nx));
        or_fr_mul(pb, pb, ch->alpha);
        or_fr_neg(pb, pb);
        or_fr_sub(pc, E4(z8, i), OR_FR_ONE);
        or_fr_mul(pc, pc, E4(l1a8, i));
        uint64_t perm[4];
        or_fr_add(perm, pa, pb);
        or_fr_add(perm, perm, pc);
        /* _compute_quotient_i (widget/lookup.cu:3-134) */
        uint64_t ct[4], la[4], lb[4], lc[4], ld[4], b0[4], b1[4], c0[4], c1[4];
        fr_copy(ct, d);
        or_fr_mul(ct, ct, ch->zeta); or_fr_add(ct, ct, c);
        or_fr_mul(ct, ct, ch->zeta); or_fr_add(ct, ct, b);
        or_fr_mul(ct, ct, ch->zeta); or_fr_add(ct, ct, a);
        or_fr_sub(la, ct, E4(f8, i));
        or_fr_mul(la, la, E4(pk->q_lookup_evals, i));
        or_fr_mul(la, la, ch->lsep);
        or_fr_add(b0, E4(f8, i), ch->eps);
        or_fr_add(b1, E4(t8, i), eopd);
        or_fr_mul(t, E4(t8, nx), ch->delta);
        or_fr_add(b1, b1, t);
        or_fr_mul(lb, E4(z28, i), opd);
        or_fr_mul(lb, lb, b0);
        or_fr_mul(lb, lb, b1);
        or_fr_mul(lb, lb, sep2);
        or_fr_add(c0, E4(h18, i), eopd);
        or_fr_mul(t, E4(h28, i), ch->delta);
        or_fr_add(c0, c0, t);
        or_fr_neg(lc, E4(z28, nx));
        or_fr_mul(lc, lc, c0);
        or_fr_add(c1, E4(h28, i), eopd);
        or_fr_mul(t, E4(h18, nx), ch->delta);
        or_fr_add(c1, c1, t);
        or_fr_mul(lc, lc, c1);
        or_fr_mul(lc, lc, sep2);
        or_fr_sub(ld, E4(z28, i), OR_FR_ONE);
        or_fr_mul(t, E4(l18, i), sep3);
        or_fr_mul(ld, ld, t);
        uint64_t lk[4];
        or_fr_add(lk, la, lb);
        or_fr_add(lk, lk, lc);
        or_fr_add(lk, lk, ld);
        /* numerator = gate + permutation + lookup (quotient.cu:360-365) */
        or_fr_add(acc, g, perm);
        or_fr_add(acc, acc, lk);
        fr_copy(E4(num, i), acc);
    }
    /* denominator = inv_mod(v_h_coset_8n); res = numerator * denominator */
    uint64_t *vh = vec_alloc(N8);
    memcpy(vh, pk->v_h_coset_8n, 32 * N8);
    or_batch_inverse(vh, N8);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)N8; i++) or_fr_mul(E4(num, i), E4(num, i), E4(vh, i));
    or_ntt(num, lg + 3, 1, 1);  /* Intt_coset */
    for (int j = 0; j < 4; j++) free(w8[j]);
    free(z8); free(pi8); free(f8); free(t8); free(h18); free(h28); free(z28);
    free(l1a); free(l1); free(l1a8); free(l18); free(vh);
    return num;
}

/* (pos, value) pairs in BTreeMap order; duplicate positions are an error
 * (PublicInputs::insert panics, pi.rs:33-38) */
typedef struct {
    uint64_t pos, v[4];
} pi_t;
static int pi_cmp(const void *a, const void *b) {
    uint64_t x = ((const pi_t *)a)->pos, y = ((const pi_t *)b)->pos;
    return x < y ? -1 : x > y;
}

static int gen_proof_impl(const CircuitC *cs, const ProverKeyC *pk, const CommitKeyC *ck,
                          uint64_t n_pi, const uint64_t *pi_pos, const uint64_t *pi_canon,
                          const char *label, int v1, ProofC *out) {
    memset(out, 0, sizeof(*out));
    uint64_t n = next_pow2(cs->n > cs->lookup_len ? cs->n : cs->lookup_len);
    uint32_t lg = lg2(n);
    uint64_t N8 = 8 * n;
    pi_t *pis = (pi_t *)calloc(n_pi ? n_pi : 1, sizeof(pi_t));
    for (uint64_t k = 0; k < n_pi; k++) {
        pis[k].pos = pi_pos[k];
        memcpy(pis[k].v, pi_canon + 4 * k, 32);
        if (pi_pos[k] >= n) { free(pis); return PNP_E_ARG; }
    }
    qsort(pis, n_pi, sizeof(pi_t), pi_cmp);
    for (uint64_t k = 1; k < n_pi; k++)
        if (pis[k].pos == pis[k - 1].pos) { free(pis); return PNP_E_ARG; }
    nz_t nz = {!all_zero(pk->q_m_evals, N8), !all_zero(pk->range_selector_evals, N8),
               !all_zero(pk->logic_selector_evals, N8),
               !all_zero(pk->fixed_group_add_selector_evals, N8),
               !all_zero(pk->variable_group_add_selector_evals, N8), !all_zero(pk->q_lookup_evals, N8)};

    challenges_t ch;
    or_transcript *tr = or_transcript_new(label);
    if (v1) {
        or_transcript_append_pi(tr, "pi", cs->pi, cs->intended_pi_pos);
    } else {
        uint64_t *pp = (uint64_t *)calloc(n_pi ? n_pi : 1, 8), *pv = vec_alloc(n_pi);
        for (uint64_t k = 0; k < n_pi; k++) { pp[k] = pis[k].pos; fr_copy(E4(pv, k), pis[k].v); }
        or_transcript_append_pis(tr, "pi", n_pi, pp, pv);
        free(pp); free(pv);
    }

    /* 1. witness polynomials (prover.rs:192-228) */
    uint64_t *wsc[4], *wpoly[4];
    const uint64_t *wsrc[4] = {cs->w_l, cs->w_r, cs->w_o, cs->w_4};
    for (int j = 0; j < 4; j++) {
        wsc[j] = pad(wsrc[j], cs->n, n);
        wpoly[j] = intt_copy(wsc[j], lg);
    }
    CommitmentC *wc[4] = {&out->a_comm, &out->b_comm, &out->c_comm, &out->d_comm};
    const char *wl[4] = {"w_l", "w_r", "w_o", "w_4"};
    for (int j = 0; j < 4; j++) commit_aff(ck, wpoly[j], n, wc[j]);
    for (int j = 0; j < 4; j++) append_comm(tr, wl[j], wc[j]);

    /* 2. lookup polynomials (prover.rs:230-329) */
    or_transcript_challenge_scalar(tr, "zeta", ch.zeta);
    or_transcript_append_scalar(tr, "zeta", ch.zeta);
    uint64_t *tc = vec_alloc(n);
    compress4(tc, pk->table1, pk->table2, pk->table3, pk->table4, ch.zeta, n);
    uint64_t *table_poly = intt_copy(tc, lg);
    uint64_t *qlk = pad(cs->q_lookup, cs->n, n);
    uint64_t *fs[4];
    for (int j = 0; j < 4; j++) fs[j] = vec_alloc(n);
    for (uint64_t i = 0; i < n; i++) {  /* query table: prover.rs:264-283 */
        if (or_fr_is_zero(E4(qlk, i))) {
            fr_copy(E4(fs[0], i), tc);
        } else {
            for (int j = 0; j < 4; j++) fr_copy(E4(fs[j], i), E4(wsc[j], i));
        }
    }
    uint64_t *fc = vec_alloc(n);
    compress4(fc, fs[0], fs[1], fs[2], fs[3], ch.zeta, n);
    uint64_t *f_poly = intt_copy(fc, lg);
    commit_aff(ck, f_poly, n, &out->f_comm);
    append_comm(tr, "f", &out->f_comm);
    uint64_t *h1 = vec_alloc(n), *h2 = vec_alloc(n);
    int rc = or_combine_split(tc, fc, n, h1, h2);  /* prover.rs:305-307 */
    if (rc != PNP_OK) {
        or_transcript_free(tr);
        for (int j = 0; j < 4; j++) { free(wsc[j]); free(wpoly[j]); free(fs[j]); }
        free(tc); free(table_poly); free(qlk); free(fc); free(f_poly); free(h1); free(h2); free(pis);
        return rc;
    }
    uint64_t *h1_poly = intt_copy(h1, lg), *h2_poly = intt_copy(h2, lg);
    commit_aff(ck, h1_poly, n, &out->h_1_comm);
    commit_aff(ck, h2_poly, n, &out->h_2_comm);
    append_comm(tr, "h1", &out->h_1_comm);
    append_comm(tr, "h2", &out->h_2_comm);

    /* 3. permutation polynomials (prover.rs:331-400) */
    or_transcript_challenge_scalar(tr, "beta", ch.beta);
    or_transcript_append_scalar(tr, "beta", ch.beta);
    or_transcript_challenge_scalar(tr, "gamma", ch.gamma);
    or_transcript_append_scalar(tr, "gamma", ch.gamma);
    or_transcript_challenge_scalar(tr, "delta", ch.delta);
    or_transcript_append_scalar(tr, "delta", ch.delta);
    or_transcript_challenge_scalar(tr, "epsilon", ch.eps);
    or_transcript_append_scalar(tr, "epsilon", ch.eps);
    uint64_t *sigc[4] = {pk->left_sigma_coeffs, pk->right_sigma_coeffs, pk->out_sigma_coeffs,
                         pk->fourth_sigma_coeffs};
    uint64_t *z_poly = permutation_poly(lg, wsc, ch.beta, ch.gamma, sigc);
    commit_aff(ck, z_poly, n, &out->z_comm);
    append_comm(tr, "z", &out->z_comm);
    uint64_t *z2_poly = or_lookup_z2(lg, fc, tc, h1, h2, ch.delta, ch.eps);
    commit_aff(ck, z2_poly, n, &out->z_2_comm);  /* not appended (prover.rs:394-397) */
    /* pi poly (pi.rs:76-86) */
    uint64_t *pie = vec_alloc(n);
    if (v1) {
        or_fr_to_mont(E4(pie, cs->intended_pi_pos), cs->pi);
    } else {
        for (uint64_t k = 0; k < n_pi; k++) or_fr_to_mont(E4(pie, pis[k].pos), pis[k].v);
    }
    uint64_t *pi_poly = intt_copy(pie, lg);

    /* 4. quotient (prover.rs:402-489) */
    or_transcript_challenge_scalar(tr, "alpha", ch.alpha);
    or_transcript_append_scalar(tr, "alpha", ch.alpha);
    or_transcript_challenge_scalar(tr, "range separation challenge", ch.range);
    or_transcript_append_scalar(tr, "range seperation challenge", ch.range);
    or_transcript_challenge_scalar(tr, "logic separation challenge", ch.logic);
    or_transcript_append_scalar(tr, "logic seperation challenge", ch.logic);
    or_transcript_challenge_scalar(tr, "fixed base separation challenge", ch.fixed);
    or_transcript_append_scalar(tr, "fixed base separation challenge", ch.fixed);
    or_transcript_challenge_scalar(tr, "variable base separation challenge", ch.var);
    or_transcript_append_scalar(tr, "variable base separation challenge", ch.var);
    or_transcript_challenge_scalar(tr, "lookup separation challenge", ch.lsep);
    or_transcript_append_scalar(tr, "lookup separation challenge", ch.lsep);
    uint64_t *t_poly = quotient_poly(lg, pk, &ch, &nz, z_poly, z2_poly, wpoly, pi_poly, f_poly,
                                     table_poly, h1_poly, h2_poly);
    CommitmentC *tcm[8] = {&out->t_1_comm, &out->t_2_comm, &out->t_3_comm, &out->t_4_comm,
                           &out->t_5_comm, &out->t_6_comm, &out->t_7_comm, &out->t_8_comm};
    for (int k = 0; k < 8; k++) commit_aff(ck, E4(t_poly, k * n), n, tcm[k]);
    for (int k = 0; k < 8; k++) {
        char lab[8];
        snprintf(lab, sizeof lab, "t_%d", k + 1);
        append_comm(tr, lab, tcm[k]);
    }

    /* 5. linearisation (linearisation_poly.rs:123-360) */
    uint64_t zc[4];
    or_transcript_challenge_scalar(tr, "z", zc);
    or_transcript_append_scalar(tr, "z", zc);
    uint64_t omega[4], zw[4], vh[4], zn[4], l1e[4], t4[4];
    or_root_of_unity(omega, lg);
    or_fr_mul(zw, zc, omega);
    or_fr_pow(vh, zc, n);
    or_fr_sub(vh, vh, OR_FR_ONE);         /* evaluate_vanishing_polynomial */
    or_fr_add(zn, vh, OR_FR_ONE);
    or_fr_from_u64(t4, n);               /* compute_first_lagrange_evaluation */
    or_fr_sub(l1e, zc, OR_FR_ONE);
    or_fr_mul(l1e, t4, l1e);
    or_fr_inv(l1e, l1e);
    or_fr_mul(l1e, vh, l1e);
    ProofEvaluationsC *ev = &out->evaluations;
    or_poly_eval(wpoly[0], n, zc, ev->wire_evals.a_eval);
    or_poly_eval(wpoly[1], n, zc, ev->wire_evals.b_eval);
    or_poly_eval(wpoly[2], n, zc, ev->wire_evals.c_eval);
    or_poly_eval(wpoly[3], n, zc, ev->wire_evals.d_eval);
    or_poly_eval(pk->left_sigma_coeffs, n, zc, ev->perm_evals.left_sigma_eval);
    or_poly_eval(pk->right_sigma_coeffs, n, zc, ev->perm_evals.right_sigma_eval);
    or_poly_eval(pk->out_sigma_coeffs, n, zc, ev->perm_evals.out_sigma_eval);
    or_poly_eval(z_poly, n, zw, ev->perm_evals.permutation_eval);
    CustomEvaluationsC *cu = &ev->custom_evals;
    or_poly_eval(pk->q_arith_coeffs, n, zc, cu->q_arith_eval);
    LookupEvaluationsC *lk = &ev->lookup_evals;
    if (nz.q_lookup) or_poly_eval(pk->q_lookup_coeffs, n, zc, lk->q_lookup_eval);
    or_poly_eval(pk->q_c_coeffs, n, zc, cu->q_c_eval);
    or_poly_eval(pk->q_l_coeffs, n, zc, cu->q_l_eval);
    or_poly_eval(pk->q_r_coeffs, n, zc, cu->q_r_eval);
    or_poly_eval(wpoly[0], n, zw, cu->a_next_eval);
    or_poly_eval(wpoly[1], n, zw, cu->b_next_eval);
    or_poly_eval(wpoly[3], n, zw, cu->d_next_eval);
    or_poly_eval(pk->q_hl_coeffs, n, zc, cu->q_hl_eval);
    or_poly_eval(pk->q_hr_coeffs, n, zc, cu->q_hr_eval);
    or_poly_eval(pk->q_h4_coeffs, n, zc, cu->q_h4_eval);
    or_poly_eval(z2_poly, n, zw, lk->z2_next_eval);
    or_poly_eval(h1_poly, n, zc, lk->h1_eval);
    or_poly_eval(h1_poly, n, zw, lk->h1_next_eval);
    or_poly_eval(h2_poly, n, zc, lk->h2_eval);
    or_poly_eval(f_poly, n, zc, lk->f_eval);
    or_poly_eval(table_poly, n, zc, lk->table_eval);
    or_poly_eval(table_poly, n, zw, lk->table_next_eval);

    const uint64_t *ae = ev->wire_evals.a_eval, *be = ev->wire_evals.b_eval,
                   *ce = ev->wire_evals.c_eval, *de = ev->wire_evals.d_eval;
    /* r(X) = sum_k S[k] P[k](X) */
    const uint64_t *P[32];
    uint64_t S[32][4], tmp[4], tmp2[4];
    int K = 0;
#define TERM(poly) (P[K] = (poly), S[K++])
    /* arithmetic (widget/arithmetic.rs:82-100) */
    const uint64_t *qae = cu->q_arith_eval;
    if (nz.q_m) { or_fr_mul(tmp, ae, be); or_fr_mul(TERM(pk->q_m_coeffs), tmp, qae); }
    or_fr_mul(TERM(pk->q_l_coeffs), ae, qae);
    or_fr_mul(TERM(pk->q_r_coeffs), be, qae);
    or_fr_mul(TERM(pk->q_o_coeffs), ce, qae);
    or_fr_mul(TERM(pk->q_4_coeffs), de, qae);
    fr_pow5(tmp, ae); or_fr_mul(TERM(pk->q_hl_coeffs), tmp, qae);
    fr_pow5(tmp, be); or_fr_mul(TERM(pk->q_hr_coeffs), tmp, qae);
    fr_pow5(tmp, de); or_fr_mul(TERM(pk->q_h4_coeffs), tmp, qae);
    fr_copy(TERM(pk->q_c_coeffs), qae);
    /* custom gates (linearisation_poly.rs:396-430): selector * constraints(evals) */
    {
        widget_vals wv = {ae, be, ce, de, cu->a_next_eval, cu->b_next_eval, cu->d_next_eval,
                          cu->q_l_eval, cu->q_r_eval, cu->q_c_eval};
        if (nz.range) or_w_range(TERM(pk->range_selector_coeffs), ch.range, &wv);
        if (nz.logic) or_w_logic(TERM(pk->logic_selector_coeffs), ch.logic, &wv);
        if (nz.fixed) or_w_fbsm(TERM(pk->fixed_group_add_selector_coeffs), ch.fixed, &wv);
        if (nz.var) or_w_cadd(TERM(pk->variable_group_add_selector_coeffs), ch.var, &wv);
    }
    /* permutation (proof_system/permutation.rs compute_linearisation) */
    {
        uint64_t bz[4], acc[4], ks[4];
        or_fr_mul(bz, ch.beta, zc);
        or_fr_add(acc, ae, bz); or_fr_add(acc, acc, ch.gamma);
        const uint64_t *wv[3] = {be, ce, de};
        const uint64_t kv[3] = {7, 13, 17};
        for (int j = 0; j < 3; j++) {
            or_fr_from_u64(ks, kv[j]);
            or_fr_mul(tmp, ks, bz);
            or_fr_add(tmp, wv[j], tmp);
            or_fr_add(tmp, tmp, ch.gamma);
            or_fr_mul(acc, acc, tmp);
        }
        or_fr_mul(acc, acc, ch.alpha);  /* identity range check */
        uint64_t a2[4], l1z[4];
        or_fr_mul(a2, ch.alpha, ch.alpha);
        or_fr_mul(l1z, l1e, a2);         /* check_is_one: l_1(z) alpha^2 */
        or_fr_add(TERM(z_poly), acc, l1z);
        /* copy range check */
        const uint64_t *sv[3] = {ev->perm_evals.left_sigma_eval, ev->perm_evals.right_sigma_eval,
                                 ev->perm_evals.out_sigma_eval};
        const uint64_t *wv2[3] = {ae, be, ce};
        fr_copy(acc, OR_FR_ONE);
        for (int j = 0; j < 3; j++) {
            or_fr_mul(tmp, ch.beta, sv[j]);
            or_fr_add(tmp, wv2[j], tmp);
            or_fr_add(tmp, tmp, ch.gamma);
            or_fr_mul(acc, acc, tmp);
        }
        or_fr_mul(tmp, ch.beta, ev->perm_evals.permutation_eval);
        or_fr_mul(acc, acc, tmp);
        or_fr_mul(acc, acc, ch.alpha);
        or_fr_neg(TERM(pk->fourth_sigma_coeffs), acc);
    }
    /* lookup (widget/lookup.rs:137-182) */
    {
        uint64_t opd[4], eopd[4], sep2[4], sep3[4], b0[4], b1[4], c1[4];
        or_fr_mul(sep2, ch.lsep, ch.lsep);
        or_fr_mul(sep3, sep2, ch.lsep);
        or_fr_add(opd, ch.delta, OR_FR_ONE);
        or_fr_mul(eopd, ch.eps, opd);
        if (nz.q_lookup) {  /* a: q_lookup (lc(a, b, c, d; zeta) - f_eval) sep */
            fr_copy(tmp, de);
            or_fr_mul(tmp, tmp, ch.zeta); or_fr_add(tmp, tmp, ce);
            or_fr_mul(tmp, tmp, ch.zeta); or_fr_add(tmp, tmp, be);
            or_fr_mul(tmp, tmp, ch.zeta); or_fr_add(tmp, tmp, ae);
            or_fr_sub(tmp, tmp, lk->f_eval);
            or_fr_mul(TERM(pk->q_lookup_coeffs), tmp, ch.lsep);
        }
        or_fr_add(b0, ch.eps, lk->f_eval);
        or_fr_add(b1, eopd, lk->table_eval);
        or_fr_mul(tmp, ch.delta, lk->table_next_eval);
        or_fr_add(b1, b1, tmp);
        or_fr_mul(tmp, l1e, sep3);                 /* b_2 */
        or_fr_mul(tmp2, opd, b0);
        or_fr_mul(tmp2, tmp2, b1);
        or_fr_mul(tmp2, tmp2, sep2);
        or_fr_add(TERM(z2_poly), tmp2, tmp);
        /* c: h1 (-z2_next sep^2)(eps(1+delta) + h2_eval + delta h1_next_eval) */
        or_fr_neg(tmp, lk->z2_next_eval);
        or_fr_mul(tmp, tmp, sep2);
        or_fr_add(c1, eopd, lk->h2_eval);
        or_fr_mul(tmp2, ch.delta, lk->h1_next_eval);
        or_fr_add(c1, c1, tmp2);
        or_fr_mul(TERM(h1_poly), tmp, c1);
    }
    /* - Z_H(z) * sum_k z^(kn) t_{k+1} (linearisation_poly.rs:311-337) */
    {
        uint64_t p[4];
        or_fr_neg(p, vh);
        for (int k = 0; k < 8; k++) {
            fr_copy(TERM(E4(t_poly, k * n)), p);
            or_fr_mul(p, p, zn);
        }
    }
#undef TERM
    uint64_t *lin = vec_alloc(n);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)n; i++) {
        uint64_t acc[4] = {0, 0, 0, 0}, t[4];
        for (int k = 0; k < K; k++) {
            or_fr_mul(t, E4(P[k], i), S[k]);
            or_fr_add(acc, acc, t);
        }
        fr_copy(E4(lin, i), acc);
    }
    /* transcript appends (prover.rs:532-572) */
    or_transcript_append_scalar(tr, "a_eval", ae);
    or_transcript_append_scalar(tr, "b_eval", be);
    or_transcript_append_scalar(tr, "c_eval", ce);
    or_transcript_append_scalar(tr, "d_eval", de);
    or_transcript_append_scalar(tr, "left_sig_eval", ev->perm_evals.left_sigma_eval);
    or_transcript_append_scalar(tr, "right_sig_eval", ev->perm_evals.right_sigma_eval);
    or_transcript_append_scalar(tr, "out_sig_eval", ev->perm_evals.out_sigma_eval);
    or_transcript_append_scalar(tr, "perm_eval", ev->perm_evals.permutation_eval);
    or_transcript_append_scalar(tr, "f_eval", lk->f_eval);
    or_transcript_append_scalar(tr, "q_lookup_eval", lk->q_lookup_eval);
    or_transcript_append_scalar(tr, "lookup_perm_eval", lk->z2_next_eval);
    or_transcript_append_scalar(tr, "h_1_eval", lk->h1_eval);
    or_transcript_append_scalar(tr, "h_1_next_eval", lk->h1_next_eval);
    or_transcript_append_scalar(tr, "h_2_eval", lk->h2_eval);
    or_transcript_append_scalar(tr, "q_arith_eval", cu->q_arith_eval);
    or_transcript_append_scalar(tr, "q_c_eval", cu->q_c_eval);
    or_transcript_append_scalar(tr, "q_l_eval", cu->q_l_eval);
    or_transcript_append_scalar(tr, "q_r_eval", cu->q_r_eval);
    or_transcript_append_scalar(tr, "q_hl_eval", cu->q_hl_eval);
    or_transcript_append_scalar(tr, "q_hr_eval", cu->q_hr_eval);
    or_transcript_append_scalar(tr, "q_h4_eval", cu->q_h4_eval);
    or_transcript_append_scalar(tr, "a_next_eval", cu->a_next_eval);
    or_transcript_append_scalar(tr, "b_next_eval", cu->b_next_eval);
    or_transcript_append_scalar(tr, "d_next_eval", cu->d_next_eval);

    /* 6. KZG openings (prover.rs:574-636, kzg10.cu:116-145) */
    uint64_t aw[4], saw[4];
    or_transcript_challenge_scalar(tr, "aggregate_witness", aw);
    const uint64_t *awp[11] = {lin, pk->left_sigma_coeffs, pk->right_sigma_coeffs,
                               pk->out_sigma_coeffs, f_poly, h2_poly, table_poly,
                               wpoly[0], wpoly[1], wpoly[2], wpoly[3]};
    uint64_t *comb = vec_alloc(n);
    {
        uint64_t pw[11][4];
        fr_copy(pw[0], OR_FR_ONE);
        for (int k = 1; k < 11; k++) or_fr_mul(pw[k], pw[k - 1], aw);
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < (int64_t)n; i++) {
            uint64_t acc[4] = {0, 0, 0, 0}, t[4];
            for (int k = 0; k < 11; k++) {
                or_fr_mul(t, E4(awp[k], i), pw[k]);
                or_fr_add(acc, acc, t);
            }
            fr_copy(E4(comb, i), acc);
        }
    }
    or_poly_div_linear(comb, n, zc);
    commit_aff(ck, comb, n, &out->aw_opening);
    or_transcript_challenge_scalar(tr, "aggregate_witness", saw);
    const uint64_t *sawp[7] = {z_poly, wpoly[0], wpoly[1], wpoly[3], h1_poly, z2_poly, table_poly};
    {
        uint64_t pw[7][4];
        fr_copy(pw[0], OR_FR_ONE);
        for (int k = 1; k < 7; k++) or_fr_mul(pw[k], pw[k - 1], saw);
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < (int64_t)n; i++) {
            uint64_t acc[4] = {0, 0, 0, 0}, t[4];
            for (int k = 0; k < 7; k++) {
                or_fr_mul(t, E4(sawp[k], i), pw[k]);
                or_fr_add(acc, acc, t);
            }
            fr_copy(E4(comb, i), acc);
        }
    }
    or_poly_div_linear(comb, n, zw);
    commit_aff(ck, comb, n, &out->saw_opening);

    or_transcript_free(tr);
    for (int j = 0; j < 4; j++) { free(wsc[j]); free(wpoly[j]); free(fs[j]); }
    free(tc); free(table_poly); free(qlk); free(fc); free(f_poly); free(h1); free(h2);
    free(h1_poly); free(h2_poly); free(z_poly); free(z2_poly); free(pie); free(pi_poly);
    free(t_poly); free(lin); free(comb); free(pis);
    return PNP_OK;
}

/* the v1 symbol (lib.rs:237-239): one public input, label "Merkle tree" */
int or_gen_proof(const CircuitC *cs, const ProverKeyC *pk, const CommitKeyC *ck, ProofC *out) {
    if (cs->intended_pi_pos >= next_pow2(cs->n > cs->lookup_len ? cs->n : cs->lookup_len))
        return PNP_E_ARG;
    return gen_proof_impl(cs, pk, ck, 1, &cs->intended_pi_pos, cs->pi, "Merkle tree", 1, out);
}

/* any number of public inputs (canonical values) and a transcript label */
int or_gen_proof_ex(const CircuitC *cs, const ProverKeyC *pk, const CommitKeyC *ck, uint64_t n_pi,
                    const uint64_t *pi_pos, const uint64_t *pi_canon, const char *label, ProofC *out) {
    return gen_proof_impl(cs, pk, ck, n_pi, pi_pos, pi_canon, label ? label : "Merkle tree", 0, out);
}
