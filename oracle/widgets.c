/*
 * oracle/widgets.c — the custom-gate constraint polynomials of the reference
 * (ZK-Garage plonk-core GateConstraint::constraints), shared by the prover
 * restatement (quotient per coset point, linearisation scalars at z) and the
 * verifier restatement (linearisation commitment scalars).
 * TEST INFRASTRUCTURE ONLY (see pnp_oracle.h).
 *   quotient term      = selector_eval(x) * constraints(sep, values at x)
 *   linearisation term = selector_poly(X) * constraints(sep, evals at z)
 * (proof_system/widget/mod.rs:83-104)
 */
#include "oracle_internal.h"

static void fr_small(uint64_t r[4], uint64_t v) { or_fr_from_u64(r, v); }
static void fr_sq(uint64_t r[4], const uint64_t a[4]) { or_fr_mul(r, a, a); }

/* delta(f) = f (f-1)(f-2)(f-3)  (widget/range.rs:66-74, logic.rs:84-93) */
static void gate_delta(uint64_t r[4], const uint64_t f[4]) {
    uint64_t k[4], t[4];
    fr_copy(r, f);
    for (uint64_t j = 1; j <= 3; j++) {
        fr_small(k, j);
        or_fr_sub(t, f, k);
        or_fr_mul(r, r, t);
    }
}

/* Range::constraints (widget/range.rs:44-60) */
void or_w_range(uint64_t out[4], const uint64_t sep[4], const widget_vals *w) {
    uint64_t four[4], kappa[4], kappa2[4], kappa3[4], t[4], u[4], acc[4];
    fr_small(four, 4);
    fr_sq(kappa, sep);
    fr_sq(kappa2, kappa);
    or_fr_mul(kappa3, kappa2, kappa);
    const uint64_t *hi[4] = {w->c, w->b, w->a, w->d_next};
    const uint64_t *lo[4] = {w->d, w->c, w->b, w->a};
    const uint64_t *kap[4] = {NULL, kappa, kappa2, kappa3};
    fr_zero(acc);
    for (int j = 0; j < 4; j++) {
        or_fr_mul(t, four, lo[j]);
        or_fr_sub(t, hi[j], t);
        gate_delta(u, t);
        if (kap[j]) or_fr_mul(u, u, kap[j]);
        or_fr_add(acc, acc, u);
    }
    or_fr_mul(out, acc, sep);
}

/* delta_xor_and (widget/logic.rs:104-133) with (a, b, w, c, q_c) */
static void delta_xor_and(uint64_t out[4], const uint64_t a[4], const uint64_t b[4],
                          const uint64_t w[4], const uint64_t c[4], const uint64_t qc[4]) {
    uint64_t k2[4], k3[4], k4[4], k9[4], k18[4], k81[4], k83[4];
    fr_small(k2, 2); fr_small(k3, 3); fr_small(k4, 4); fr_small(k9, 9);
    fr_small(k18, 18); fr_small(k81, 81); fr_small(k83, 83);
    uint64_t apb[4], t[4], u[4], F[4], E[4], B[4];
    or_fr_add(apb, a, b);
    /* F = w (w (4w - 18(a+b) + 81) + 18(a^2 + b^2) - 81(a+b) + 83) */
    or_fr_mul(t, k4, w);
    or_fr_mul(u, k18, apb);
    or_fr_sub(t, t, u);
    or_fr_add(t, t, k81);
    or_fr_mul(t, w, t);
    uint64_t a2[4], b2[4];
    fr_sq(a2, a);
    fr_sq(b2, b);
    or_fr_add(u, a2, b2);
    or_fr_mul(u, k18, u);
    or_fr_add(t, t, u);
    or_fr_mul(u, k81, apb);
    or_fr_sub(t, t, u);
    or_fr_add(t, t, k83);
    or_fr_mul(F, w, t);
    /* E = 3(a+b+c) - 2F */
    or_fr_add(t, apb, c);
    or_fr_mul(E, k3, t);
    or_fr_mul(u, k2, F);
    or_fr_sub(E, E, u);
    /* B = q_c (9c - 3(a+b)) */
    or_fr_mul(t, k9, c);
    or_fr_mul(u, k3, apb);
    or_fr_sub(t, t, u);
    or_fr_mul(B, qc, t);
    or_fr_add(out, B, E);
}

/* Logic::constraints (widget/logic.rs:59-82) */
void or_w_logic(uint64_t out[4], const uint64_t sep[4], const widget_vals *w) {
    uint64_t four[4], kappa[4], kappa2[4], kappa3[4], kappa4[4];
    fr_small(four, 4);
    fr_sq(kappa, sep);
    fr_sq(kappa2, kappa);
    or_fr_mul(kappa3, kappa2, kappa);
    or_fr_mul(kappa4, kappa3, kappa);
    uint64_t a[4], b[4], d[4], t[4], c0[4], c1[4], c2[4], c3[4], c4[4], acc[4];
    or_fr_mul(t, four, w->a); or_fr_sub(a, w->a_next, t);
    gate_delta(c0, a);
    or_fr_mul(t, four, w->b); or_fr_sub(b, w->b_next, t);
    gate_delta(c1, b); or_fr_mul(c1, c1, kappa);
    or_fr_mul(t, four, w->d); or_fr_sub(d, w->d_next, t);
    gate_delta(c2, d); or_fr_mul(c2, c2, kappa2);
    or_fr_mul(t, a, b); or_fr_sub(c3, w->c, t); or_fr_mul(c3, c3, kappa3);
    delta_xor_and(c4, a, b, w->c, d, w->q_c); or_fr_mul(c4, c4, kappa4);
    or_fr_add(acc, c0, c1);
    or_fr_add(acc, acc, c2);
    or_fr_add(acc, acc, c3);
    or_fr_add(acc, acc, c4);
    or_fr_mul(out, acc, sep);
}

/* Jubjub (ark-ed-on-bls12-381) a = -1, d = -(10240/10241); the reference
 * GPU path's constants, lib/PLONK/src/bls12_381/edwards.cu:5-33 (Montgomery) */
static const uint64_t COEFF_A[4] = {18446744060824649731ULL, 18102478225614246908ULL,
                                    11073656695919314959ULL, 6613806504683796440ULL};
static const uint64_t COEFF_D[4] = {3049539848285517488ULL, 18189135023605205683ULL,
                                    8793554888777148625ULL, 6339087681201251886ULL};

/* FixedBaseScalarMul::constraints (widget/ecc/fixed_base_scalar_mul.rs:89-155) */
void or_w_fbsm(uint64_t out[4], const uint64_t sep[4], const widget_vals *w) {
    uint64_t kappa[4], kappa2[4], kappa3[4], one[4], t[4], u[4];
    fr_copy(one, OR_FR_ONE);
    fr_sq(kappa, sep);
    fr_sq(kappa2, kappa);
    or_fr_mul(kappa3, kappa2, kappa);
    /* bit = d_next - 2 d */
    uint64_t bit[4], bitc[4], bm1[4], bp1[4];
    or_fr_sub(bit, w->d_next, w->d);
    or_fr_sub(bit, bit, w->d);
    or_fr_sub(bm1, bit, one);
    or_fr_add(bp1, bit, one);
    or_fr_mul(bitc, bit, bm1);
    or_fr_mul(bitc, bitc, bp1);
    /* y_alpha = bit^2 (y_beta - 1) + 1, x_alpha = x_beta bit */
    uint64_t ya[4], xa[4];
    fr_sq(t, bit);
    or_fr_sub(u, w->q_r, one);
    or_fr_mul(ya, t, u);
    or_fr_add(ya, ya, one);
    or_fr_mul(xa, w->q_l, bit);
    /* xy_consistency = (bit q_c - xy_alpha) kappa, xy_alpha = c */
    uint64_t xyc[4];
    or_fr_mul(xyc, bit, w->q_c);
    or_fr_sub(xyc, xyc, w->c);
    or_fr_mul(xyc, xyc, kappa);
    /* common = xy_alpha acc_x acc_y D */
    uint64_t m[4];
    or_fr_mul(m, w->c, w->a);
    or_fr_mul(m, m, w->b);
    or_fr_mul(m, m, COEFF_D);
    /* x: lhs = x3 + x3 m, rhs = x_alpha acc_y + y_alpha acc_x */
    uint64_t lhs[4], rhs[4], xac[4], yac[4];
    or_fr_mul(t, w->a_next, m);
    or_fr_add(lhs, w->a_next, t);
    or_fr_mul(rhs, xa, w->b);
    or_fr_mul(t, ya, w->a);
    or_fr_add(rhs, rhs, t);
    or_fr_sub(xac, lhs, rhs);
    or_fr_mul(xac, xac, kappa2);
    /* y: lhs = y3 - y3 m, rhs = y_alpha acc_y - A x_alpha acc_x */
    or_fr_mul(t, w->b_next, m);
    or_fr_sub(lhs, w->b_next, t);
    or_fr_mul(rhs, ya, w->b);
    or_fr_mul(t, COEFF_A, xa);
    or_fr_mul(t, t, w->a);
    or_fr_sub(rhs, rhs, t);
    or_fr_sub(yac, lhs, rhs);
    or_fr_mul(yac, yac, kappa3);
    uint64_t acc[4];
    or_fr_add(acc, bitc, xac);
    or_fr_add(acc, acc, yac);
    or_fr_add(acc, acc, xyc);
    or_fr_mul(out, acc, sep);
}

/* CurveAddition::constraints (widget/ecc/curve_addition.rs:61-96) */
void or_w_cadd(uint64_t out[4], const uint64_t sep[4], const widget_vals *w) {
    const uint64_t *x1 = w->a, *x3 = w->a_next, *y1 = w->b, *y3 = w->b_next, *x2 = w->c, *y2 = w->d,
                   *x1y2 = w->d_next;
    uint64_t kappa[4], kappa2[4], t[4], u[4];
    fr_sq(kappa, sep);
    fr_sq(kappa2, kappa);
    uint64_t xyc[4], y1x2[4], y1y2[4], x1x2[4];
    or_fr_mul(xyc, x1, y2);
    or_fr_sub(xyc, xyc, x1y2);
    or_fr_mul(y1x2, y1, x2);
    or_fr_mul(y1y2, y1, y2);
    or_fr_mul(x1x2, x1, x2);
    uint64_t dm[4];  /* D x1y2 y1x2 */
    or_fr_mul(dm, COEFF_D, x1y2);
    or_fr_mul(dm, dm, y1x2);
    uint64_t x3c[4], y3c[4];
    or_fr_add(t, x1y2, y1x2);           /* x3_lhs */
    or_fr_mul(u, x3, dm);
    or_fr_add(u, x3, u);                /* x3_rhs */
    or_fr_sub(x3c, t, u);
    or_fr_mul(x3c, x3c, kappa);
    or_fr_mul(t, COEFF_A, x1x2);
    or_fr_sub(t, y1y2, t);              /* y3_lhs */
    or_fr_mul(u, y3, dm);
    or_fr_sub(u, y3, u);                /* y3_rhs */
    or_fr_sub(y3c, t, u);
    or_fr_mul(y3c, y3c, kappa2);
    uint64_t acc[4];
    or_fr_add(acc, xyc, x3c);
    or_fr_add(acc, acc, y3c);
    or_fr_mul(out, acc, sep);
}

