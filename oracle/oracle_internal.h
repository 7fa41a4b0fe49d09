/* oracle/oracle_internal.h — shared helpers of the CPU restatement.
 * TEST INFRASTRUCTURE ONLY (see pnp_oracle.h). */
#ifndef ORACLE_INTERNAL_H
#define ORACLE_INTERNAL_H
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include "pnp_oracle.h"
#ifdef _OPENMP
#include <omp.h>
#endif

typedef unsigned __int128 u128;

extern const uint64_t OR_FR_P[4], OR_FR_ONE[4], OR_FR_R2[4], OR_FR_ROOT32[4], OR_FR_GEN[4];
extern const uint64_t OR_FQ_P[6], OR_FQ_ONE[6], OR_FQ_R2[6];

static inline void fr_copy(uint64_t *r, const uint64_t *a) { memcpy(r, a, 32); }
static inline void fq_copy(uint64_t *r, const uint64_t *a) { memcpy(r, a, 48); }
static inline void fr_zero(uint64_t *r) { memset(r, 0, 32); }

void or_fr_neg(uint64_t r[4], const uint64_t a[4]);
int or_fr_is_zero(const uint64_t a[4]);
int or_fr_eq(const uint64_t a[4], const uint64_t b[4]);
void or_fr_from_u64(uint64_t r[4], uint64_t x);
void or_fq_neg(uint64_t r[6], const uint64_t a[6]);
int or_fq_is_zero(const uint64_t a[6]);
int or_fq_eq(const uint64_t a[6], const uint64_t b[6]);
int or_gt_n(const uint64_t *a, const uint64_t *b, int N);

/* root of unity of order 2^lg (domain.cu:29-36), Montgomery */
void or_root_of_unity(uint64_t r[4], uint32_t lg);

/* Jacobian G1 point (X, Y, Z), Montgomery; Z = 0 is infinity */
typedef struct { uint64_t x[6], y[6], z[6]; } or_g1j;
void or_g1j_set_inf(or_g1j *p);
int or_g1j_is_inf(const or_g1j *p);
void or_g1j_double(or_g1j *r, const or_g1j *p);
void or_g1j_add(or_g1j *r, const or_g1j *p, const or_g1j *q);
void or_g1j_add_affine(or_g1j *r, const or_g1j *p, const uint64_t aff[12]);
void or_g1j_to_affine(uint64_t aff[12], const or_g1j *p);
void or_g1_msm(or_g1j *r, const uint64_t *points, const uint64_t *scalars_canon, uint64_t n);

/* custom-gate constraints (widgets.c): wire values a..d, the next-row values
 * and the q_l / q_r / q_c selector values at one point */
typedef struct {
    const uint64_t *a, *b, *c, *d;
    const uint64_t *a_next, *b_next, *d_next, *q_l, *q_r, *q_c;
} widget_vals;
void or_w_range(uint64_t out[4], const uint64_t sep[4], const widget_vals *w);
void or_w_logic(uint64_t out[4], const uint64_t sep[4], const widget_vals *w);
void or_w_fbsm(uint64_t out[4], const uint64_t sep[4], const widget_vals *w);
uint64_t *or_lookup_z2(uint32_t lg, const uint64_t *f, const uint64_t *t, const uint64_t *h1,
                       const uint64_t *h2, const uint64_t delta[4], const uint64_t eps[4]);
void or_w_cadd(uint64_t out[4], const uint64_t sep[4], const widget_vals *w);

#endif
