/*
 * pnp_oracle.h — CPU restatement of the reference gen_proof path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (the HIP library under
 * zprize23-gpu-submission_amd/) includes, links or calls this code; only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
 * oracle/liboracle.so, and only as the checker / CPU baseline.
 *
 * Every function cites the reference file:line whose semantics it restates
 * (paths relative to /root/reference/Prize 1B/plonk-core/).  The restatement
 * is pinned by tests/golden/ fixtures generated from blst and STROBE compiled
 * from the reference's own sources (oracle/ref.mk -> oracle/_ref/).
 */
#ifndef PNP_ORACLE_H
#define PNP_ORACLE_H

#include <stdint.h>
#include <stddef.h>
#include "../include/pnp_plonk.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- field: lib/PLONK/utils/mont/cuda/ff/bls12-381.hpp:7-93 ---- */
void or_fr_add(uint64_t r[4], const uint64_t a[4], const uint64_t b[4]);
void or_fr_sub(uint64_t r[4], const uint64_t a[4], const uint64_t b[4]);
void or_fr_mul(uint64_t r[4], const uint64_t a[4], const uint64_t b[4]);
void or_fr_inv(uint64_t r[4], const uint64_t a[4]);
void or_fr_to_mont(uint64_t r[4], const uint64_t a[4]);
void or_fr_from_mont(uint64_t r[4], const uint64_t a[4]);
void or_fr_pow(uint64_t r[4], const uint64_t a[4], uint64_t e);
void or_fq_add(uint64_t r[6], const uint64_t a[6], const uint64_t b[6]);
void or_fq_sub(uint64_t r[6], const uint64_t a[6], const uint64_t b[6]);
void or_fq_mul(uint64_t r[6], const uint64_t a[6], const uint64_t b[6]);
void or_fq_inv(uint64_t r[6], const uint64_t a[6]);
void or_fq_to_mont(uint64_t r[6], const uint64_t a[6]);
void or_fq_from_mont(uint64_t r[6], const uint64_t a[6]);

/* ---- vectors of Fr (n elements, 4 limbs each) ---- */
void or_fr_vec_to_mont(uint64_t *v, uint64_t n);
void or_fr_vec_from_mont(uint64_t *v, uint64_t n);

/* ---- NTT: zksnark_ntt.cu:74-92 / ntt.cuh:57-144 / domain.cu:12-36 ---- */
void or_ntt(uint64_t *v, uint32_t lg_n, int inverse, int coset);
void or_coset_lde8(const uint64_t *coeffs, uint64_t *out8, uint32_t lg_n);

/* ---- polynomial helpers: function.cu:162-173, mont_arithmetic.cu:305-360 ---- */
void or_poly_eval(const uint64_t *c, uint64_t n, const uint64_t x[4], uint64_t out[4]);
void or_poly_div_linear(uint64_t *p, uint64_t n, const uint64_t z[4]);
void or_prefix_product(uint64_t *v, uint64_t n);
void or_batch_inverse(uint64_t *v, uint64_t n);

/* ---- G1: PLONK/src/point.cu, zkp/cuda/ec/jacobian_t.hpp ---- */
/* affine points are 12 u64 (x, y) Montgomery; inf as (0, one). */
void or_g1_generator(uint64_t out_aff[12]);
void or_g1_add_affine(uint64_t out[12], const uint64_t a[12], const uint64_t b[12]);
void or_g1_mul(uint64_t out[12], const uint64_t p[12], const uint64_t scalar_canon[4]);
/* d_out[i] = tau^i * G (affine) */
void or_srs(uint64_t *out, uint64_t n, const uint64_t tau_mont[4]);
/* commit (kzg10.cu:31-44): scalars Montgomery, result affine Montgomery */
void or_commit(const uint64_t *points, const uint64_t *scalars_mont, uint64_t n,
               uint64_t out_aff[12]);

/* ---- transcript: transcript.cuh:21-73, strobe.cpp, serialize.cuh ---- */
typedef struct or_transcript or_transcript;
or_transcript *or_transcript_new(const char *label);
void or_transcript_free(or_transcript *t);
void or_transcript_append_message(or_transcript *t, const char *label,
                                  const uint8_t *msg, size_t len);
void or_transcript_append_scalar(or_transcript *t, const char *label, const uint64_t s_mont[4]);
void or_transcript_append_point(or_transcript *t, const char *label, const uint64_t aff[12]);
void or_transcript_append_pi(or_transcript *t, const char *label,
                             const uint64_t pi_canon[4], uint64_t pos);
/* several public inputs, positions strictly increasing (BTreeMap order) */
void or_transcript_append_pis(or_transcript *t, const char *label, uint64_t k,
                              const uint64_t *pos, const uint64_t *vals_canon);
void or_transcript_challenge_bytes(or_transcript *t, const char *label, uint8_t *out, size_t len);
void or_transcript_challenge_scalar(or_transcript *t, const char *label, uint64_t out_mont[4]);
/* raw state for fixtures: 200 B strobe state + pos, pos_begin, cur_flags */
void or_transcript_state(const or_transcript *t, uint8_t st[200], int meta[3]);
/* raw keccak-f[1600] (strobe.cpp keccak_p) */
void or_keccak_f1600(uint64_t st[25]);

/* ---- full prover: gen_proof.cuh:10-489 ---- */
int or_gen_proof(const CircuitC *cs, const ProverKeyC *pk, const CommitKeyC *ck, ProofC *out);
/* prover.rs semantics with n_pi public inputs (positions, canonical values;
 * any order, zeros dropped) and a transcript label */
int or_gen_proof_ex(const CircuitC *cs, const ProverKeyC *pk, const CommitKeyC *ck, uint64_t n_pi,
                    const uint64_t *pi_pos, const uint64_t *pi_canon, const char *label, ProofC *out);
/* plookup: MultiSet::combine_split (multiset.rs:131) of t (n) and f (n) into
 * h1, h2 (n each); PNP_E_ARG when a value of f is not in t */
int or_combine_split(const uint64_t *t, const uint64_t *f, uint64_t n, uint64_t *h1, uint64_t *h2);

/* ---- verifier: proof.rs:123-431 (Proof::verify), circuit.rs:325-344 ---- */
/* commitments to the preprocessed polynomials, affine Montgomery, infinity
 * = (0, Fq one); g = powers_of_g[0] (the KZG verifier key's G) */
#define OR_VK_POLYS 23
typedef struct {
    uint64_t n;
    uint64_t g[12];
    uint64_t q_m[12], q_l[12], q_r[12], q_o[12], q_4[12], q_c[12], q_hl[12], q_hr[12], q_h4[12],
        q_arith[12];
    uint64_t range[12], logic[12], fixed_group_add[12], variable_group_add[12];
    uint64_t left_sigma[12], right_sigma[12], out_sigma[12], fourth_sigma[12];
    uint64_t q_lookup[12], table_1[12], table_2[12], table_3[12], table_4[12];
} or_verifier_key;
/* slots in the order q_m, q_l, q_r, q_o, q_4, q_c, q_hl, q_hr, q_h4, q_arith,
 * range, logic, fixed_group_add, variable_group_add, left/right/out/fourth
 * sigma, q_lookup, table_1..4 */
void or_vk_slots(or_verifier_key *vk, uint64_t (*dst[OR_VK_POLYS])[12]);
void or_verifier_key_from_coeffs(or_verifier_key *vk, uint64_t n, const uint64_t *srs,
                                 const uint64_t *const coeffs[OR_VK_POLYS]);
/* the same key from the trapdoor: commit(p) = [p(tau)] G (g_aff = SRS_0) */
void or_verifier_key_tau(or_verifier_key *vk, uint64_t n, const uint64_t g_aff[12],
                         const uint64_t *const coeffs[OR_VK_POLYS], const uint64_t tau_mont[4]);
/* the two KZG openings reduced to G1: out = {L_aw, W_aw, L_saw, W_saw} with
 * L = sum ch^i C_i - (sum ch^i v_i) G + x W; accept iff e(L, H) = e(W, [tau]H) */
int or_verify_kzg_points(const or_verifier_key *vk, const ProofC *p, const char *label,
                         uint64_t n_pi, const uint64_t *pi_pos, const uint64_t *pi_canon,
                         uint64_t out[4][12]);
/* 1 = accept, 0 = reject; the pairing check decided with the SRS trapdoor
 * (L == tau W) */
int or_verify(const or_verifier_key *vk, const ProofC *p, const char *label, uint64_t n_pi,
              const uint64_t *pi_pos, const uint64_t *pi_canon, const uint64_t tau_mont[4]);

/* ---- synthetic instances: CPU mirror of csrc/synth.hip (inputs, not reference) ---- */
void or_synth_random_fr(uint64_t *d, uint64_t n, uint64_t seed);
void or_synth_circuit(uint64_t *const w[4], uint64_t *const sel[9], uint64_t *const sigma[4],
                      uint64_t n, uint64_t ng, uint64_t pi_pos, const uint64_t pi_canon[4]);
void or_synth_coset_consts(uint64_t *vh, uint64_t *x, uint32_t lg);
/* pnp_synth_merkle: the reference's Poseidon Merkle circuit of `height`;
 * pc_mont = 199 Montgomery constants (rk[189], MDS row-major, tag) */
int or_synth_merkle(uint32_t height, const uint64_t *pc_mont, const uint64_t *leaves, const uint64_t *blind,
                    uint64_t *nodes, uint64_t *const w[4], uint64_t *const sel[9], uint64_t *const sigma[4],
                    uint64_t n, uint64_t root_canon[4]);

/* threads used by the OpenMP loops (for cpu_baseline.cores) */
int or_num_threads(void);
void or_set_num_threads(int t);

#ifdef __cplusplus
}
#endif
#endif
