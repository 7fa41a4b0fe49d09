/*
 * oracle/verifier.c — CPU restatement of the reference PLONK verifier.
 * TEST INFRASTRUCTURE ONLY (see pnp_oracle.h).
 *
 * Restates Proof::verify (plonk-core/src/proof_system/proof.rs:123-431) as
 * driven by verify_proof (plonk-core/src/circuit.rs:325-344) and the
 * merkle-tree driver (merkle-tree/src/main.rs:106-140): a fresh transcript
 * with the caller's label, the public inputs appended as their BTreeMap, the
 * transcript replayed to recover every challenge, r_0 (proof.rs:433-494),
 * the linearisation commitment (proof.rs:497-598 with the widget
 * VerifierKeys: widget/arithmetic.rs:154-199, widget/range.rs:44-60,
 * widget/logic.rs:59-121, widget/ecc/fixed_base_scalar_mul.rs:89-155,
 * widget/ecc/curve_addition.rs:61-96, widget/lookup.rs:238-294,
 * proof_system/permutation.rs:327-385) and the two batched KZG checks
 * (SonicKZG10::check of ark-poly-commit 0.3, commitment.rs:22).
 *
 * The pairing-product check of SonicKZG10, e(C - vG + zW, H) = e(W, [tau]H),
 * is reduced here to the two G1 points (L = C - vG + zW, W) of each opening:
 *   - or_verify_kzg_points() returns them, so a test can run the pairing
 *     itself (blst_miller_loop / blst_final_exp of the reference's own blst,
 *     oracle/_ref/libpairing_ref.so);
 *   - or_verify() decides with the SRS trapdoor tau (L = tau W), which needs
 *     no pairing and is exactly equivalent because e(., H) is injective.
 * Commitments equal to (0, Fq one) are the point at infinity (the flags
 * main.rs:112-123 sets by hand for f, h1, h2, t7, t8 are computed here).
 */
#include "oracle_internal.h"

typedef struct {
    or_g1j acc;
} lc_t;

static void lc_init(lc_t *l) { or_g1j_set_inf(&l->acc); }
/* acc += s * P (s Montgomery Fr, P affine) */
static void lc_add(lc_t *l, const uint64_t s_mont[4], const uint64_t P[12]) {
    uint64_t c[4], t[12];
    or_fr_from_mont(c, s_mont);
    or_g1_mul(t, P, c);
    or_g1j_add_affine(&l->acc, &l->acc, t);
}

static void fr_pow5(uint64_t r[4], const uint64_t a[4]) {
    uint64_t a2[4], a4[4];
    or_fr_mul(a2, a, a);
    or_fr_mul(a4, a2, a2);
    or_fr_mul(r, a4, a);
}
static void fr_small(uint64_t r[4], uint64_t v) { or_fr_from_u64(r, v); }
static void fr_sq(uint64_t r[4], const uint64_t a[4]) { or_fr_mul(r, a, a); }

static void comm_aff(uint64_t aff[12], const CommitmentC *c) {
    memcpy(aff, c->x, 48);
    memcpy(aff + 6, c->y, 48);
}

/* compute_first_lagrange_evaluation (proof.rs:619-630) */
static void l1_eval(uint64_t out[4], uint64_t n, const uint64_t zh[4], const uint64_t z[4]) {
    uint64_t nf[4], t[4];
    or_fr_from_u64(nf, n);
    or_fr_sub(t, z, OR_FR_ONE);
    or_fr_mul(t, nf, t);
    or_fr_inv(t, t);
    or_fr_mul(out, zh, t);
}

/* compute_barycentric_eval (proof.rs:632-674) over the PI map */
static void pi_eval(uint64_t out[4], uint64_t n, uint32_t lg, const uint64_t zh[4], const uint64_t z[4],
                    uint64_t k, const uint64_t *pos, const uint64_t *vals_mont) {
    uint64_t nf[4], ninv[4], num[4], w[4], winv[4], acc[4];
    or_fr_from_u64(nf, n);
    or_fr_inv(ninv, nf);
    or_fr_mul(num, zh, ninv);
    or_root_of_unity(w, lg);
    or_fr_inv(winv, w);
    fr_zero(acc);
    for (uint64_t i = 0; i < k; i++) {
        if (or_fr_is_zero(vals_mont + 4 * i)) continue;
        uint64_t d[4];
        or_fr_pow(d, winv, pos[i]);
        or_fr_mul(d, d, z);
        or_fr_sub(d, d, OR_FR_ONE);
        or_fr_inv(d, d);
        or_fr_mul(d, d, vals_mont + 4 * i);
        or_fr_add(acc, acc, d);
    }
    or_fr_mul(out, acc, num);
}

static void append_comm(or_transcript *t, const char *label, const CommitmentC *c) {
    uint64_t aff[12];
    comm_aff(aff, c);
    or_transcript_append_point(t, label, aff);
}

/* Sum_i ch^i C_i and Sum_i ch^i v_i; then L = C - v G + z W (SonicKZG10::check) */
static void kzg_point(uint64_t L[12], uint64_t W[12], const uint64_t (*comms)[12],
                      const uint64_t (*evals)[4], int k, const uint64_t ch[4], const uint64_t z[4],
                      const CommitmentC *w, const uint64_t g[12]) {
    lc_t l;
    lc_init(&l);
    uint64_t p[4], v[4], t[4];
    fr_copy(p, OR_FR_ONE);
    fr_zero(v);
    for (int i = 0; i < k; i++) {
        lc_add(&l, p, comms[i]);
        or_fr_mul(t, evals[i], p);
        or_fr_add(v, v, t);
        or_fr_mul(p, p, ch);
    }
    comm_aff(W, w);
    or_fr_neg(t, v);
    lc_add(&l, t, g);       /* - v G */
    lc_add(&l, z, W);       /* + z W */
    or_g1j_to_affine(L, &l.acc);
}

int or_verify_kzg_points(const or_verifier_key *vk, const ProofC *p, const char *label, uint64_t n_pi,
                         const uint64_t *pi_pos, const uint64_t *pi_canon, uint64_t out[4][12]) {
    const uint64_t n = vk->n;
    uint32_t lg = 0;
    while ((1ULL << lg) < n) lg++;
    if ((1ULL << lg) != n) return PNP_E_ARG;
    for (uint64_t i = 0; i < n_pi; i++)
        if (pi_pos[i] >= n || (i && pi_pos[i] <= pi_pos[i - 1])) return PNP_E_ARG;  /* BTreeMap order */
    uint64_t *pi_m = (uint64_t *)calloc(n_pi ? n_pi : 1, 32);
    for (uint64_t i = 0; i < n_pi; i++) or_fr_to_mont(pi_m + 4 * i, pi_canon + 4 * i);

    or_transcript *tr = or_transcript_new(label);
    or_transcript_append_pis(tr, "pi", n_pi, pi_pos, pi_canon);
    append_comm(tr, "w_l", &p->a_comm);
    append_comm(tr, "w_r", &p->b_comm);
    append_comm(tr, "w_o", &p->c_comm);
    append_comm(tr, "w_4", &p->d_comm);
    uint64_t zeta[4], beta[4], gamma[4], delta[4], eps[4], alpha[4];
    uint64_t range_c[4], logic_c[4], fixed_c[4], var_c[4], lsep[4], zc[4];
    or_transcript_challenge_scalar(tr, "zeta", zeta);
    or_transcript_append_scalar(tr, "zeta", zeta);
    append_comm(tr, "f", &p->f_comm);
    append_comm(tr, "h1", &p->h_1_comm);
    append_comm(tr, "h2", &p->h_2_comm);
    or_transcript_challenge_scalar(tr, "beta", beta);
    or_transcript_append_scalar(tr, "beta", beta);
    or_transcript_challenge_scalar(tr, "gamma", gamma);
    or_transcript_append_scalar(tr, "gamma", gamma);
    or_transcript_challenge_scalar(tr, "delta", delta);
    or_transcript_append_scalar(tr, "delta", delta);
    or_transcript_challenge_scalar(tr, "epsilon", eps);
    or_transcript_append_scalar(tr, "epsilon", eps);
    if (or_fr_eq(beta, gamma) || or_fr_eq(beta, delta) || or_fr_eq(beta, eps) ||
        or_fr_eq(gamma, delta) || or_fr_eq(gamma, eps) || or_fr_eq(delta, eps)) {
        or_transcript_free(tr);
        free(pi_m);
        return PNP_E_ARG;  /* proof.rs:192-197 asserts */
    }
    append_comm(tr, "z", &p->z_comm);
    or_transcript_challenge_scalar(tr, "alpha", alpha);
    or_transcript_append_scalar(tr, "alpha", alpha);
    or_transcript_challenge_scalar(tr, "range separation challenge", range_c);
    or_transcript_append_scalar(tr, "range seperation challenge", range_c);
    or_transcript_challenge_scalar(tr, "logic separation challenge", logic_c);
    or_transcript_append_scalar(tr, "logic seperation challenge", logic_c);
    or_transcript_challenge_scalar(tr, "fixed base separation challenge", fixed_c);
    or_transcript_append_scalar(tr, "fixed base separation challenge", fixed_c);
    or_transcript_challenge_scalar(tr, "variable base separation challenge", var_c);
    or_transcript_append_scalar(tr, "variable base separation challenge", var_c);
    or_transcript_challenge_scalar(tr, "lookup separation challenge", lsep);
    or_transcript_append_scalar(tr, "lookup separation challenge", lsep);
    const CommitmentC *tcm[8] = {&p->t_1_comm, &p->t_2_comm, &p->t_3_comm, &p->t_4_comm,
                                 &p->t_5_comm, &p->t_6_comm, &p->t_7_comm, &p->t_8_comm};
    static const char *tl[8] = {"t_1", "t_2", "t_3", "t_4", "t_5", "t_6", "t_7", "t_8"};
    for (int k = 0; k < 8; k++) append_comm(tr, tl[k], tcm[k]);
    or_transcript_challenge_scalar(tr, "z", zc);
    or_transcript_append_scalar(tr, "z", zc);

    uint64_t zh[4], zn[4], l1[4], t[4], u[4];
    or_fr_pow(zn, zc, n);
    or_fr_sub(zh, zn, OR_FR_ONE);
    l1_eval(l1, n, zh, zc);

    const ProofEvaluationsC *ev = &p->evaluations;
    const uint64_t *ae = ev->wire_evals.a_eval, *be = ev->wire_evals.b_eval,
                   *ce = ev->wire_evals.c_eval, *de = ev->wire_evals.d_eval;
    const uint64_t *s1 = ev->perm_evals.left_sigma_eval, *s2 = ev->perm_evals.right_sigma_eval,
                   *s3 = ev->perm_evals.out_sigma_eval, *zhat = ev->perm_evals.permutation_eval;
    const LookupEvaluationsC *lk = &ev->lookup_evals;
    const CustomEvaluationsC *cu = &ev->custom_evals;
    uint64_t opd[4], eopd[4], sep2[4], sep3[4], alpha2[4];
    or_fr_add(opd, OR_FR_ONE, delta);
    or_fr_mul(eopd, eps, opd);
    fr_sq(sep2, lsep);
    or_fr_mul(sep3, sep2, lsep);
    fr_sq(alpha2, alpha);

    /* r_0 (proof.rs:433-494) */
    uint64_t r0[4];
    {
        uint64_t pie[4], b[4], c[4], d[4], e[4];
        pi_eval(pie, n, lg, zh, zc, n_pi, pi_pos, pi_m);
        const uint64_t *wv[3] = {ae, be, ce}, *sv[3] = {s1, s2, s3};
        fr_copy(b, OR_FR_ONE);
        for (int j = 0; j < 3; j++) {
            or_fr_mul(t, beta, sv[j]);
            or_fr_add(t, wv[j], t);
            or_fr_add(t, t, gamma);
            or_fr_mul(b, b, t);
        }
        or_fr_add(t, de, gamma);
        or_fr_mul(t, t, zhat);
        or_fr_mul(t, t, alpha);
        or_fr_mul(b, b, t);
        or_fr_mul(c, l1, alpha2);
        uint64_t d0[4], d1[4], d2[4];
        or_fr_mul(d0, sep2, lk->z2_next_eval);
        or_fr_mul(t, delta, lk->h2_eval);
        or_fr_add(d1, eopd, t);
        or_fr_add(d2, eopd, lk->h2_eval);
        or_fr_mul(t, delta, lk->h1_next_eval);
        or_fr_add(d2, d2, t);
        or_fr_mul(d, d0, d1);
        or_fr_mul(d, d, d2);
        or_fr_mul(e, sep3, l1);
        or_fr_sub(r0, pie, b);
        or_fr_sub(r0, r0, c);
        or_fr_sub(r0, r0, d);
        or_fr_sub(r0, r0, e);
    }

    /* evaluations into the transcript (proof.rs:227-279), custom evals in
     * the order util::to_proof_evaluations gives them (util.rs:246-256) */
    or_transcript_append_scalar(tr, "a_eval", ae);
    or_transcript_append_scalar(tr, "b_eval", be);
    or_transcript_append_scalar(tr, "c_eval", ce);
    or_transcript_append_scalar(tr, "d_eval", de);
    or_transcript_append_scalar(tr, "left_sig_eval", s1);
    or_transcript_append_scalar(tr, "right_sig_eval", s2);
    or_transcript_append_scalar(tr, "out_sig_eval", s3);
    or_transcript_append_scalar(tr, "perm_eval", zhat);
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

    /* linearisation commitment (proof.rs:497-598) */
    uint64_t lin[12];
    {
        lc_t l;
        lc_init(&l);
        const uint64_t *qa = cu->q_arith_eval;
        /* arithmetic (widget/arithmetic.rs:154-199) */
        or_fr_mul(t, ae, be); or_fr_mul(t, t, qa); lc_add(&l, t, vk->q_m);
        or_fr_mul(t, ae, qa); lc_add(&l, t, vk->q_l);
        or_fr_mul(t, be, qa); lc_add(&l, t, vk->q_r);
        or_fr_mul(t, de, qa); lc_add(&l, t, vk->q_4);
        or_fr_mul(t, ce, qa); lc_add(&l, t, vk->q_o);
        fr_pow5(t, ae); or_fr_mul(t, t, qa); lc_add(&l, t, vk->q_hl);
        fr_pow5(t, be); or_fr_mul(t, t, qa); lc_add(&l, t, vk->q_hr);
        fr_pow5(t, de); or_fr_mul(t, t, qa); lc_add(&l, t, vk->q_h4);
        lc_add(&l, qa, vk->q_c);
        /* custom gates (widget/mod.rs:109-130) */
        widget_vals wv = {ae, be, ce, de, cu->a_next_eval, cu->b_next_eval, cu->d_next_eval,
                          cu->q_l_eval, cu->q_r_eval, cu->q_c_eval};
        or_w_range(t, range_c, &wv); lc_add(&l, t, vk->range);
        or_w_logic(t, logic_c, &wv); lc_add(&l, t, vk->logic);
        or_w_fbsm(t, fixed_c, &wv); lc_add(&l, t, vk->fixed_group_add);
        or_w_cadd(t, var_c, &wv); lc_add(&l, t, vk->variable_group_add);
        /* lookup (widget/lookup.rs:238-294) */
        {
            uint64_t comp[4], a[4], b0[4], b1[4], b[4], c0[4], c1[4], c[4], aff[12];
            fr_copy(comp, de);  /* lc([a, b, c, d], zeta) = a + zeta b + zeta^2 c + zeta^3 d */
            or_fr_mul(comp, comp, zeta); or_fr_add(comp, comp, ce);
            or_fr_mul(comp, comp, zeta); or_fr_add(comp, comp, be);
            or_fr_mul(comp, comp, zeta); or_fr_add(comp, comp, ae);
            or_fr_sub(a, comp, lk->f_eval);
            or_fr_mul(a, a, lsep);
            lc_add(&l, a, vk->q_lookup);
            or_fr_add(b0, eps, lk->f_eval);
            or_fr_add(b1, eopd, lk->table_eval);
            or_fr_mul(t, delta, lk->table_next_eval);
            or_fr_add(b1, b1, t);
            or_fr_mul(b, opd, b0);
            or_fr_mul(b, b, b1);
            or_fr_mul(b, b, sep2);
            or_fr_mul(t, l1, sep3);
            or_fr_add(b, b, t);
            comm_aff(aff, &p->z_2_comm);
            lc_add(&l, b, aff);
            or_fr_neg(c0, lk->z2_next_eval);
            or_fr_mul(c0, c0, sep2);
            or_fr_add(c1, eopd, lk->h2_eval);
            or_fr_mul(t, delta, lk->h1_next_eval);
            or_fr_add(c1, c1, t);
            or_fr_mul(c, c0, c1);
            comm_aff(aff, &p->h_1_comm);
            lc_add(&l, c, aff);
        }
        /* permutation (proof_system/permutation.rs:327-385) */
        {
            uint64_t bz[4], x[4], y[4], k[4], aff[12];
            or_fr_mul(bz, beta, zc);
            or_fr_add(x, ae, bz);
            or_fr_add(x, x, gamma);
            const uint64_t *wv2[3] = {be, ce, de};
            const uint64_t kv[3] = {7, 13, 17};
            for (int j = 0; j < 3; j++) {
                fr_small(k, kv[j]);
                or_fr_mul(t, bz, k);
                or_fr_add(t, wv2[j], t);
                or_fr_add(t, t, gamma);
                if (j == 2) or_fr_mul(t, t, alpha);
                or_fr_mul(x, x, t);
            }
            or_fr_mul(t, l1, alpha2);
            or_fr_add(x, x, t);
            comm_aff(aff, &p->z_comm);
            lc_add(&l, x, aff);
            const uint64_t *wv3[3] = {ae, be, ce}, *sv[3] = {s1, s2, s3};
            fr_copy(y, OR_FR_ONE);
            for (int j = 0; j < 3; j++) {
                or_fr_mul(t, beta, sv[j]);
                or_fr_add(t, wv3[j], t);
                or_fr_add(t, t, gamma);
                or_fr_mul(y, y, t);
            }
            or_fr_mul(t, beta, zhat);
            or_fr_mul(t, t, alpha);
            or_fr_mul(y, y, t);
            or_fr_neg(y, y);
            lc_add(&l, y, vk->fourth_sigma);
        }
        /* quotient chunks: -Z_H(z) z^(kn) (proof.rs:572-596) */
        {
            uint64_t s[4], aff[12];
            or_fr_neg(s, zh);
            for (int k = 0; k < 8; k++) {
                comm_aff(aff, tcm[k]);
                lc_add(&l, s, aff);
                or_fr_mul(s, s, zn);
            }
        }
        or_g1j_to_affine(lin, &l.acc);
    }

    /* table commitment t1 + zeta t2 + zeta^2 t3 + zeta^3 t4 (proof.rs:301-310) */
    uint64_t table[12];
    {
        lc_t l;
        lc_init(&l);
        fr_copy(t, OR_FR_ONE);
        const uint64_t *tb[4] = {vk->table_1, vk->table_2, vk->table_3, vk->table_4};
        for (int j = 0; j < 4; j++) {
            lc_add(&l, t, tb[j]);
            or_fr_mul(t, t, zeta);
        }
        or_g1j_to_affine(table, &l.acc);
    }

    uint64_t aw[4], saw[4];
    or_transcript_challenge_scalar(tr, "aggregate_witness", aw);
    or_transcript_challenge_scalar(tr, "aggregate_witness", saw);
    or_transcript_free(tr);

    uint64_t comms[11][12], evals[11][4];
    /* aggregate witness at z (proof.rs:333-360) */
    memcpy(comms[0], lin, 96);
    memcpy(comms[1], vk->left_sigma, 96);
    memcpy(comms[2], vk->right_sigma, 96);
    memcpy(comms[3], vk->out_sigma, 96);
    comm_aff(comms[4], &p->f_comm);
    comm_aff(comms[5], &p->h_2_comm);
    memcpy(comms[6], table, 96);
    comm_aff(comms[7], &p->a_comm);
    comm_aff(comms[8], &p->b_comm);
    comm_aff(comms[9], &p->c_comm);
    comm_aff(comms[10], &p->d_comm);
    or_fr_neg(evals[0], r0);
    fr_copy(evals[1], s1);
    fr_copy(evals[2], s2);
    fr_copy(evals[3], s3);
    fr_copy(evals[4], lk->f_eval);
    fr_copy(evals[5], lk->h2_eval);
    fr_copy(evals[6], lk->table_eval);
    fr_copy(evals[7], ae);
    fr_copy(evals[8], be);
    fr_copy(evals[9], ce);
    fr_copy(evals[10], de);
    uint64_t g[12];
    memcpy(g, vk->g, 96);
    kzg_point(out[0], out[1], (const uint64_t(*)[12])comms, (const uint64_t(*)[4])evals, 11, aw, zc,
              &p->aw_opening, g);
    /* shifted aggregate witness at z w (proof.rs:362-381) */
    comm_aff(comms[0], &p->z_comm);
    comm_aff(comms[1], &p->a_comm);
    comm_aff(comms[2], &p->b_comm);
    comm_aff(comms[3], &p->d_comm);
    comm_aff(comms[4], &p->h_1_comm);
    comm_aff(comms[5], &p->z_2_comm);
    memcpy(comms[6], table, 96);
    fr_copy(evals[0], zhat);
    fr_copy(evals[1], cu->a_next_eval);
    fr_copy(evals[2], cu->b_next_eval);
    fr_copy(evals[3], cu->d_next_eval);
    fr_copy(evals[4], lk->h1_next_eval);
    fr_copy(evals[5], lk->z2_next_eval);
    fr_copy(evals[6], lk->table_next_eval);
    uint64_t w[4], zw[4];
    or_root_of_unity(w, lg);
    or_fr_mul(zw, zc, w);
    kzg_point(out[2], out[3], (const uint64_t(*)[12])comms, (const uint64_t(*)[4])evals, 7, saw, zw,
              &p->saw_opening, g);
    (void)u;
    free(pi_m);
    return PNP_OK;
}

int or_verify(const or_verifier_key *vk, const ProofC *p, const char *label, uint64_t n_pi,
              const uint64_t *pi_pos, const uint64_t *pi_canon, const uint64_t tau_mont[4]) {
    uint64_t pts[4][12];
    int rc = or_verify_kzg_points(vk, p, label, n_pi, pi_pos, pi_canon, pts);
    if (rc != PNP_OK) return 0;
    uint64_t tc[4], tw[12];
    or_fr_from_mont(tc, tau_mont);
    for (int k = 0; k < 2; k++) {
        or_g1_mul(tw, pts[2 * k + 1], tc);  /* tau W */
        if (memcmp(tw, pts[2 * k], 96) != 0) return 0;
    }
    return 1;
}

/* verifier key = commitments to the preprocessed polynomials
 * (preprocess.rs, widget VerifierKeys); coefficient pointers may be NULL
 * for all-zero polynomials (empty Rust Vecs). */
void or_verifier_key_from_coeffs(or_verifier_key *vk, uint64_t n, const uint64_t *srs,
                                 const uint64_t *const coeffs[OR_VK_POLYS]) {
    vk->n = n;
    memcpy(vk->g, srs, 96);
    uint64_t(*dst[OR_VK_POLYS])[12];
    or_vk_slots(vk, dst);
    for (int k = 0; k < OR_VK_POLYS; k++) {
        if (!coeffs[k]) {
            memset(dst[k][0], 0, 48);
            fq_copy(dst[k][0] + 6, OR_FQ_ONE);
        } else {
            or_commit(srs, coeffs[k], n, dst[k][0]);
        }
    }
}

/* The same verifier key from the SRS trapdoor: SRS_i = [tau^i] G, so
 * commit(p) = sum_i p_i [tau^i] G = [p(tau)] G — one Horner evaluation and one
 * scalar multiplication per polynomial instead of an n-point MSM (a checker
 * for instances whose tau is known, e.g. bench.py's). */
void or_verifier_key_tau(or_verifier_key *vk, uint64_t n, const uint64_t g_aff[12],
                         const uint64_t *const coeffs[OR_VK_POLYS], const uint64_t tau_mont[4]) {
    vk->n = n;
    memcpy(vk->g, g_aff, 96);
    uint64_t(*dst[OR_VK_POLYS])[12];
    or_vk_slots(vk, dst);
#pragma omp parallel for schedule(dynamic, 1)
    for (int k = 0; k < OR_VK_POLYS; k++) {
        if (!coeffs[k]) {
            memset(dst[k][0], 0, 48);
            fq_copy(dst[k][0] + 6, OR_FQ_ONE);
            continue;
        }
        uint64_t acc[4] = {0, 0, 0, 0};
        for (uint64_t i = n; i-- > 0;) {
            or_fr_mul(acc, acc, tau_mont);
            or_fr_add(acc, acc, coeffs[k] + 4 * i);
        }
        or_commit(g_aff, acc, 1, dst[k][0]);
    }
}

void or_vk_slots(or_verifier_key *vk, uint64_t (*dst[OR_VK_POLYS])[12]) {
    uint64_t(*s[OR_VK_POLYS])[12] = {
        &vk->q_m, &vk->q_l, &vk->q_r, &vk->q_o, &vk->q_4, &vk->q_c, &vk->q_hl, &vk->q_hr, &vk->q_h4,
        &vk->q_arith, &vk->range, &vk->logic, &vk->fixed_group_add, &vk->variable_group_add,
        &vk->left_sigma, &vk->right_sigma, &vk->out_sigma, &vk->fourth_sigma, &vk->q_lookup,
        &vk->table_1, &vk->table_2, &vk->table_3, &vk->table_4};
    for (int k = 0; k < OR_VK_POLYS; k++) dst[k] = s[k];
}
