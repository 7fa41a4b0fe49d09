// protocol.h — argument blocks and launchers of the fused gen_proof passes
// (protocol.hip).  Argument structs are passed by value as kernel arguments.
#pragma once
#include "pnp_internal.h"

namespace pnp {

__host__ __device__ inline Fr from_u64_limbs_dev(const uint64_t *l) {
    Fr r;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        r.v[2 * i] = (uint32_t)l[i];
        r.v[2 * i + 1] = (uint32_t)(l[i] >> 32);
    }
    return r;
}

struct PermArgs {
    const uint64_t *w[4];
    const uint64_t *sigma[4];  // sigma evaluations on the n-domain
    Fr bk[4];                  // beta * k_j, k = 1, 7, 13, 17
    Fr beta, gamma, omega;
    const uint64_t *tw;  // w^e, e < max(n/2, 1): the NTT's forward twiddles (ntt_twiddles)
};

// nullptr arrays are known-zero and not read, except z28: nullptr means the
// lookup-trivial case z2 = 1 with f = t = h1 = h2 = 0, in which every z2 term of
// the lookup quotient cancels exactly; q_m / q_lookup nullptr = zero selector.
struct QuotArgs {
    const uint64_t *w8[4], *z8, *pi8, *f8, *t8, *h18, *h28, *z28, *l18;
    const uint64_t *q_m, *q_l, *q_r, *q_o, *q_4, *q_c, *q_hl, *q_hr, *q_h4, *q_arith, *q_lookup;
    const uint64_t *sig[4], *lin, *vh_inv;
    // closed forms on the standard coset (pnp_ctx::pk_std_coset), replacing
    // pi8 / l18: l1v = L1 / Z_H = n^-1 / (x - 1), pinv = 1 / (x - w^pos),
    // PI / Z_H = c_pi * pinv with c_pi = pi * w^pos / n
    const uint64_t *l1v, *pinv;
    Fr c_pi;
    uint64_t n;     // block length: arrays are in block-bitrev layout
    uint32_t lg_n;  // (point 8j + m -> m n + brev(j), ntt.hip lde_blocks)
    Fr alpha, alpha2, beta, gamma, delta, eps, zeta, lsep;
    Fr bk[4], opd, eopd, sep2, sep3;
};

// k_quotient29: the quotient of the common case (no custom gates, no lookup,
// the standard coset: the Merkle circuit) in radix-2^29
// arithmetic (fr29.cuh).  The arrays marked 2^261 hold values in that
// Montgomery form (the wire / z LDEs through the scaled twist, lde_blocks
// form29; key copies made at load); vh_inv, l1v and pinv stay in the 2^256
// form, so the final products return the quotient to it.  Constants: nine
// 29-bit limbs of their 2^261 forms (fr_to_r29_limbs).
struct Quot29Args {
    const uint64_t *w8[4], *z8, *pi8;  // 2^261 (pi8: several PIs, nullptr otherwise)
    const uint64_t *q_m, *q_l, *q_r, *q_o, *q_4, *q_c, *q_hl, *q_hr, *q_h4, *q_arith;  // 2^261
    const uint64_t *sig[4], *lin;                                                // 2^261
    const uint64_t *vh_inv, *l1v, *pinv;                                         // 2^256
    uint32_t c_pi[9], alpha[9], alpha2[9], beta[9], gamma[9], one[9];
    uint64_t n;
    uint32_t lg_n;
};
// the 2^261 form of a (2^256-form) Fr as nine 29-bit limbs, canonical
void fr_to_r29_limbs(const Fr &a, uint32_t l[9]);
void k_quotient29(const Quot29Args &q, uint64_t N8, uint64_t *out, hipStream_t s);
// out = 32 in (mod r) elementwise: 2^256-form arrays -> their 2^261 forms
void k_to_form29(const uint64_t *in, uint64_t *out, uint64_t n, hipStream_t s);

// custom-gate quotient terms (k_widgets): block-layout arrays as QuotArgs;
// sel = range, logic, fixed-base scalar mul, curve addition selector
// evaluations (nullptr = zero selector), sep = their separation challenges
struct WidgetArgs {
    const uint64_t *w8[4], *q_l, *q_r, *q_c, *vh_inv;
    const uint64_t *sel[4];
    Fr sep[4];
    uint64_t n;
    uint32_t lg_n;
};

constexpr int LIN_MAX = 32;
struct LinArgs {
    int k;
    const uint64_t *p[LIN_MAX];
    Fr s[LIN_MAX];
};

void k_compress4(uint64_t *out, const uint64_t *t0, const uint64_t *t1, const uint64_t *t2,
                 const uint64_t *t3, const Fr &z, uint64_t n, hipStream_t s);
void k_query_f(uint64_t *out, const uint64_t *ql, uint64_t n_gates, const uint64_t *const w[4],
               const uint64_t *tc, const Fr &z, uint64_t n, hipStream_t s);
void k_perm_numden(uint64_t *num, uint64_t *den, const PermArgs &a, uint64_t n, hipStream_t s);
void k_lookup_nd(uint64_t *num, uint64_t *den, const uint64_t *f, const uint64_t *t,
                 const uint64_t *h1, const uint64_t *h2, const Fr &delta, const Fr &eps, uint64_t n,
                 hipStream_t s);
void k_mul_inplace(uint64_t *a, const uint64_t *b, uint64_t n, hipStream_t s);
bool k_any_nonzero(const uint64_t *v, uint64_t words, DevBuf &scratch, hipStream_t s);
void k_any_nonzero_n(const uint64_t *v, uint64_t words, uint64_t stride, int cnt, bool *nz, DevBuf &scratch,
                     hipStream_t s);
// any word of a differs from b
bool k_any_diff(const uint64_t *a, const uint64_t *b, uint64_t words, DevBuf &scratch, hipStream_t s);
// 128-bit content hash of `words` u64 in HBM (synchronous)
void k_hash_words(const uint64_t *a, uint64_t words, DevBuf &scratch, hipStream_t s, uint64_t out[2]);
// strided affine points (x / y: 6 u64 each at x_off / y_off, an infinity byte
// at inf_off, `stride` bytes per point) -> packed 12-u64 points; false when a
// point is flagged infinity (synchronous)
bool k_pack_affine(const uint8_t *src, uint64_t n, uint64_t stride, uint64_t x_off, uint64_t y_off,
                   uint64_t inf_off, uint64_t *dst, DevBuf &scratch, hipStream_t s);
// out_i = a * in_i + b
void k_affine(uint64_t *out, const uint64_t *in, const Fr &a, const Fr &b, uint64_t n, hipStream_t s);
void k_quotient(const QuotArgs &q, uint64_t N8, uint64_t *out, hipStream_t s);
void k_lincomb(const LinArgs &a, uint64_t n, uint64_t *out, hipStream_t s);
void k_widgets(const WidgetArgs &g, uint64_t N8, uint64_t *out, hipStream_t s);
// MultiSet::combine_split (lookup/multiset.rs:131-180) of the compressed table
// t and query f (n each, Montgomery) into h1, h2 (n each); false when a value
// of f does not occur in t (lookup.hip)
bool combine_split(pnp_ctx *ctx, const uint64_t *t, const uint64_t *f, uint64_t n, uint64_t *h1,
                   uint64_t *h2, hipStream_t s);
// empty kernel marking the start of a proof in kernel traces
void k_proof_marker(hipStream_t s);

}  // namespace pnp
