/*
 * oracle/g1.c — BLS12-381 G1 arithmetic and MSM (CPU restatement).
 * TEST INFRASTRUCTURE ONLY (see pnp_oracle.h).
 *
 * Restates: PLONK/src/point.cu:29-257 (to_affine, add_assign, double,
 * add_assign_mixed — Jacobian, a = 0), the MSM contract of
 * utils/function.cu:275-290 + PLONK/src/arithmetic.cu:105-127 (sum s_i P_i over
 * min(#points, #scalars) terms, canonical scalars) and commit()
 * (KZG/kzg10.cu:31-44: to_base, MSM, mix with the empty hiding commitment,
 * to_affine; infinity -> (0, Fq one)).  The MSM algorithm here is a plain
 * unsigned-window Pippenger; any correct MSM yields the same affine point.
 */
#include "oracle_internal.h"

/* BLS12-381 G1 generator, canonical coordinates */
static const uint64_t G1_X[6] = {0xfb3af00adb22c6bbULL, 0x6c55e83ff97a1aefULL,
                                 0xa14e3a3f171bac58ULL, 0xc3688c4f9774b905ULL,
                                 0x2695638c4fa9ac0fULL, 0x17f1d3a73197d794ULL};
static const uint64_t G1_Y[6] = {0x0caa232946c5e7e1ULL, 0xd03cc744a2888ae4ULL,
                                 0x00db18cb2c04b3edULL, 0xfcf5e095d5d00af6ULL,
                                 0xa09e30ed741d8ae4ULL, 0x08b3f481e3aaa0f1ULL};

void or_g1_generator(uint64_t out_aff[12]) {
    or_fq_to_mont(out_aff, G1_X);
    or_fq_to_mont(out_aff + 6, G1_Y);
}

void or_g1j_set_inf(or_g1j *p) {
    fq_copy(p->x, OR_FQ_ONE);
    fq_copy(p->y, OR_FQ_ONE);
    memset(p->z, 0, 48);
}
int or_g1j_is_inf(const or_g1j *p) { return or_fq_is_zero(p->z); }

static int aff_is_inf(const uint64_t a[12]) {
    /* AffinePointG1::is_zero (point.cu:5-15): x == 0 and y == one */
    return or_fq_is_zero(a) && or_fq_eq(a + 6, OR_FQ_ONE);
}

/* double_ProjectivePointG1 (point.cu:121-183), dbl-2009-l */
void or_g1j_double(or_g1j *r, const or_g1j *p) {
    if (or_g1j_is_inf(p)) { *r = *p; return; }
    uint64_t A[6], B[6], C[6], D[6], E[6], F[6], t[6], x3[6], y3[6], z3[6];
    or_fq_mul(A, p->x, p->x);
    or_fq_mul(B, p->y, p->y);
    or_fq_mul(C, B, B);
    or_fq_add(t, p->x, B);
    or_fq_mul(t, t, t);
    or_fq_sub(t, t, A);
    or_fq_sub(t, t, C);
    or_fq_add(D, t, t);
    or_fq_add(E, A, A);
    or_fq_add(E, E, A);
    or_fq_mul(F, E, E);
    or_fq_mul(z3, p->y, p->z);
    or_fq_add(z3, z3, z3);
    or_fq_sub(x3, F, D);
    or_fq_sub(x3, x3, D);
    or_fq_sub(t, D, x3);
    or_fq_mul(y3, E, t);
    or_fq_add(C, C, C);
    or_fq_add(C, C, C);
    or_fq_add(C, C, C);
    or_fq_sub(y3, y3, C);
    fq_copy(r->x, x3);
    fq_copy(r->y, y3);
    fq_copy(r->z, z3);
}

/* add_assign (point.cu:49-119), add-2007-bl */
void or_g1j_add(or_g1j *r, const or_g1j *p, const or_g1j *q) {
    if (or_g1j_is_inf(p)) { *r = *q; return; }
    if (or_g1j_is_inf(q)) { *r = *p; return; }
    uint64_t z1z1[6], z2z2[6], u1[6], u2[6], s1[6], s2[6], h[6], i[6], j[6], rr[6], v[6], t[6];
    or_fq_mul(z1z1, p->z, p->z);
    or_fq_mul(z2z2, q->z, q->z);
    or_fq_mul(u1, p->x, z2z2);
    or_fq_mul(u2, q->x, z1z1);
    or_fq_mul(s1, p->y, q->z);
    or_fq_mul(s1, s1, z2z2);
    or_fq_mul(s2, q->y, p->z);
    or_fq_mul(s2, s2, z1z1);
    if (or_fq_eq(u1, u2)) {
        if (or_fq_eq(s1, s2)) { or_g1j_double(r, p); return; }
        or_g1j_set_inf(r);
        return;
    }
    or_fq_sub(h, u2, u1);
    or_fq_add(i, h, h);
    or_fq_mul(i, i, i);
    or_fq_mul(j, h, i);
    or_fq_sub(rr, s2, s1);
    or_fq_add(rr, rr, rr);
    or_fq_mul(v, u1, i);
    or_g1j out;
    or_fq_mul(out.x, rr, rr);
    or_fq_sub(out.x, out.x, j);
    or_fq_sub(out.x, out.x, v);
    or_fq_sub(out.x, out.x, v);
    or_fq_sub(t, v, out.x);
    or_fq_mul(out.y, rr, t);
    or_fq_mul(t, s1, j);
    or_fq_add(t, t, t);
    or_fq_sub(out.y, out.y, t);
    or_fq_add(t, p->z, q->z);
    or_fq_mul(t, t, t);
    or_fq_sub(t, t, z1z1);
    or_fq_sub(t, t, z2z2);
    or_fq_mul(out.z, t, h);
    *r = out;
}

/* add_assign_mixed (point.cu:184-257), madd-2007-bl */
void or_g1j_add_affine(or_g1j *r, const or_g1j *p, const uint64_t aff[12]) {
    if (aff_is_inf(aff)) { *r = *p; return; }
    if (or_g1j_is_inf(p)) {
        fq_copy(r->x, aff);
        fq_copy(r->y, aff + 6);
        fq_copy(r->z, OR_FQ_ONE);
        return;
    }
    uint64_t z1z1[6], u2[6], s2[6], h[6], hh[6], i[6], j[6], rr[6], v[6], t[6];
    or_fq_mul(z1z1, p->z, p->z);
    or_fq_mul(u2, aff, z1z1);
    or_fq_mul(s2, aff + 6, p->z);
    or_fq_mul(s2, s2, z1z1);
    if (or_fq_eq(p->x, u2)) {
        if (or_fq_eq(p->y, s2)) { or_g1j_double(r, p); return; }
        or_g1j_set_inf(r);
        return;
    }
    or_fq_sub(h, u2, p->x);
    or_fq_mul(hh, h, h);
    or_fq_add(i, hh, hh);
    or_fq_add(i, i, i);
    or_fq_mul(j, h, i);
    or_fq_sub(rr, s2, p->y);
    or_fq_add(rr, rr, rr);
    or_fq_mul(v, p->x, i);
    or_g1j out;
    or_fq_mul(out.x, rr, rr);
    or_fq_sub(out.x, out.x, j);
    or_fq_sub(out.x, out.x, v);
    or_fq_sub(out.x, out.x, v);
    or_fq_sub(t, v, out.x);
    or_fq_mul(out.y, rr, t);
    or_fq_mul(t, p->y, j);
    or_fq_add(t, t, t);
    or_fq_sub(out.y, out.y, t);
    or_fq_add(t, p->z, h);
    or_fq_mul(t, t, t);
    or_fq_sub(t, t, z1z1);
    or_fq_sub(out.z, t, hh);
    *r = out;
}

/* to_affine (point.cu:29-47) */
void or_g1j_to_affine(uint64_t aff[12], const or_g1j *p) {
    if (or_g1j_is_inf(p)) {
        memset(aff, 0, 48);
        fq_copy(aff + 6, OR_FQ_ONE);
        return;
    }
    uint64_t zi[6], zi2[6], zi3[6];
    or_fq_inv(zi, p->z);
    or_fq_mul(zi2, zi, zi);
    or_fq_mul(zi3, zi2, zi);
    or_fq_mul(aff, p->x, zi2);
    or_fq_mul(aff + 6, p->y, zi3);
}

void or_g1_add_affine(uint64_t out[12], const uint64_t a[12], const uint64_t b[12]) {
    or_g1j p;
    or_g1j_set_inf(&p);
    or_g1j_add_affine(&p, &p, a);
    or_g1j_add_affine(&p, &p, b);
    or_g1j_to_affine(out, &p);
}

static void g1j_mul(or_g1j *r, const uint64_t p[12], const uint64_t s[4]) {
    or_g1j acc;
    or_g1j_set_inf(&acc);
    for (int b = 255; b >= 0; b--) {
        or_g1j_double(&acc, &acc);
        if ((s[b / 64] >> (b % 64)) & 1) or_g1j_add_affine(&acc, &acc, p);
    }
    *r = acc;
}

void or_g1_mul(uint64_t out[12], const uint64_t p[12], const uint64_t scalar_canon[4]) {
    or_g1j r;
    g1j_mul(&r, p, scalar_canon);
    or_g1j_to_affine(out, &r);
}

void or_srs(uint64_t *out, uint64_t n, const uint64_t tau_mont[4]) {
    uint64_t g[12];
    or_g1_generator(g);
    const int64_t CH = 64;
#pragma omp parallel for schedule(dynamic)
    for (int64_t c = 0; c < (int64_t)((n + CH - 1) / CH); c++) {
        uint64_t start = (uint64_t)c * CH, end = start + CH < n ? start + CH : n;
        uint64_t tp[4], canon[4];
        or_fr_pow(tp, tau_mont, start);
        for (uint64_t i = start; i < end; i++) {
            or_fr_from_mont(canon, tp);
            or_g1_mul(out + 12 * i, g, canon);
            or_fr_mul(tp, tp, tau_mont);
        }
    }
}

static int msm_window(uint64_t n) {
    int c = 1;
    while ((1ULL << (c + 1)) * (uint64_t)(c + 1) < n) c++;  /* ~ log2(n) - log2(log2 n) */
    if (c > 16) c = 16;
    return c;
}

void or_g1_msm(or_g1j *r, const uint64_t *points, const uint64_t *scalars_canon, uint64_t n) {
    int c = msm_window(n);
    int nw = (255 + c - 1) / c;
    uint64_t nb = (1ULL << c) - 1;
    or_g1j *win = (or_g1j *)malloc(sizeof(or_g1j) * nw);
#pragma omp parallel for schedule(dynamic)
    for (int w = 0; w < nw; w++) {
        or_g1j *bk = (or_g1j *)malloc(sizeof(or_g1j) * nb);
        for (uint64_t b = 0; b < nb; b++) or_g1j_set_inf(&bk[b]);
        int bit = w * c;
        for (uint64_t i = 0; i < n; i++) {
            const uint64_t *s = scalars_canon + 4 * i;
            uint64_t d = 0;
            for (int k = 0; k < c && bit + k < 256; k++)
                d |= ((s[(bit + k) / 64] >> ((bit + k) % 64)) & 1ULL) << k;
            if (d) or_g1j_add_affine(&bk[d - 1], &bk[d - 1], points + 12 * i);
        }
        or_g1j run, sum;
        or_g1j_set_inf(&run);
        or_g1j_set_inf(&sum);
        for (int64_t b = (int64_t)nb - 1; b >= 0; b--) {
            or_g1j_add(&run, &run, &bk[b]);
            or_g1j_add(&sum, &sum, &run);
        }
        win[w] = sum;
        free(bk);
    }
    or_g1j acc;
    or_g1j_set_inf(&acc);
    for (int w = nw - 1; w >= 0; w--) {
        for (int k = 0; k < c; k++) or_g1j_double(&acc, &acc);
        or_g1j_add(&acc, &acc, &win[w]);
    }
    *r = acc;
    free(win);
}

void or_commit(const uint64_t *points, const uint64_t *scalars_mont, uint64_t n,
               uint64_t out_aff[12]) {
    uint64_t *canon = (uint64_t *)malloc(32 * (n ? n : 1));
    memcpy(canon, scalars_mont, 32 * n);
    or_fr_vec_from_mont(canon, n);
    or_g1j r;
    or_g1_msm(&r, points, canon, n);
    or_g1j_to_affine(out_aff, &r);
    free(canon);
}
