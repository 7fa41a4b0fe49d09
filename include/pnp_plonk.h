/*
 * pnp_plonk.h — C-ABI boundary of the MI355X gen_proof backend.
 *
 * Drop-in replacement for the reference's CUDA library behind the Rust FFI:
 *   Rust declaration   : plonk-core/src/lib.rs:52-239   (repr(C) structs + extern "C" gen_proof)
 *   C implementation   : plonk-core/lib/hello.cu:4-6     (gen_proof -> prove)
 *   C struct mirror    : plonk-core/lib/PLONK/src/structure.cuh:7-329
 * (paths relative to /root/reference/Prize 1B/).
 *
 * Everything in section 1 is layout-identical to lib.rs, so the Rust host
 * links this library instead of libzprize without source changes
 * (see INTEGRATION.md).  Sections 2-4 are additive (v2) entry points: explicit
 * lengths, error codes, resident (HBM) keys and the operator API used by the
 * parity tests.  No torch or HIP types appear in any signature.
 *
 * Field encodings (identical to arkworks 0.3 / the reference):
 *   Fr  : 4 x u64 little-endian limbs, Montgomery form R = 2^256 mod r
 *   Fq  : 6 x u64 little-endian limbs, Montgomery form R = 2^384 mod q
 *   G1 affine point: {Fq x, Fq y} (12 u64), no infinity flag;
 *   the point at infinity is reported as x = 0, y = Fq::one (Montgomery),
 *   as the reference's to_affine (PLONK/src/point.cu:29-47).
 */
#ifndef PNP_PLONK_H
#define PNP_PLONK_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ */
/* 1. v1 ABI — byte-for-byte the reference FFI (lib.rs:52-239)         */
/* ------------------------------------------------------------------ */

/* lib.rs:53-59 */
typedef struct {
    uint64_t a_eval[4];
    uint64_t b_eval[4];
    uint64_t c_eval[4];
    uint64_t d_eval[4];
} WireEvaluationsC;

/* lib.rs:61-67 */
typedef struct {
    uint64_t left_sigma_eval[4];
    uint64_t right_sigma_eval[4];
    uint64_t out_sigma_eval[4];
    uint64_t permutation_eval[4];
} PermutationEvaluationsC;

/* lib.rs:69-81 */
typedef struct {
    uint64_t q_arith_eval[4];
    uint64_t q_c_eval[4];
    uint64_t q_l_eval[4];
    uint64_t q_r_eval[4];
    uint64_t q_hl_eval[4];
    uint64_t q_hr_eval[4];
    uint64_t q_h4_eval[4];
    uint64_t a_next_eval[4];
    uint64_t b_next_eval[4];
    uint64_t d_next_eval[4];
} CustomEvaluationsC;

/* lib.rs:101-111 */
typedef struct {
    uint64_t q_lookup_eval[4];
    uint64_t z2_next_eval[4];
    uint64_t h1_eval[4];
    uint64_t h1_next_eval[4];
    uint64_t h2_eval[4];
    uint64_t f_eval[4];
    uint64_t table_eval[4];
    uint64_t table_next_eval[4];
} LookupEvaluationsC;

/* lib.rs:112-118 */
typedef struct {
    WireEvaluationsC wire_evals;
    PermutationEvaluationsC perm_evals;
    LookupEvaluationsC lookup_evals;
    CustomEvaluationsC custom_evals;
} ProofEvaluationsC;

/* lib.rs:231-235 : affine G1, Montgomery Fq limbs */
typedef struct {
    uint64_t x[6];
    uint64_t y[6];
} CommitmentC;

/* lib.rs:120-142 */
typedef struct {
    CommitmentC a_comm;
    CommitmentC b_comm;
    CommitmentC c_comm;
    CommitmentC d_comm;
    CommitmentC z_comm;
    CommitmentC f_comm;
    CommitmentC h_1_comm;
    CommitmentC h_2_comm;
    CommitmentC z_2_comm;
    CommitmentC t_1_comm;
    CommitmentC t_2_comm;
    CommitmentC t_3_comm;
    CommitmentC t_4_comm;
    CommitmentC t_5_comm;
    CommitmentC t_6_comm;
    CommitmentC t_7_comm;
    CommitmentC t_8_comm;
    CommitmentC aw_opening;
    CommitmentC saw_opening;
    ProofEvaluationsC evaluations;
} ProofC;

/* lib.rs:144-155.  n = unpadded gate count; q_lookup/w_* hold n Montgomery Fr;
 * pi holds ONE Fr in canonical (non-Montgomery) form (prover.rs:717-725). */
typedef struct {
    uint64_t n;
    uint64_t lookup_len;
    uint64_t intended_pi_pos;
    uint64_t *q_lookup;
    uint64_t *pi;
    uint64_t *w_l;
    uint64_t *w_r;
    uint64_t *w_o;
    uint64_t *w_4;
} CircuitC;

/* lib.rs:157-223.  With D = next_pow2(max(n, lookup_len)):
 *   *_coeffs, table1..4 : D Montgomery Fr
 *   *_evals, linear_evaluations, v_h_coset_8n : 8*D Montgomery Fr
 * The coeff buffers of q_m, the four custom-gate selectors and q_lookup are
 * empty Rust Vecs for the Merkle circuit and are never read (gen_proof.cuh:277,
 * 319-329), exactly as in the reference. */
typedef struct {
    uint64_t *q_m_coeffs;
    uint64_t *q_m_evals;
    uint64_t *q_l_coeffs;
    uint64_t *q_l_evals;
    uint64_t *q_r_coeffs;
    uint64_t *q_r_evals;
    uint64_t *q_o_coeffs;
    uint64_t *q_o_evals;
    uint64_t *q_4_coeffs;
    uint64_t *q_4_evals;
    uint64_t *q_c_coeffs;
    uint64_t *q_c_evals;
    uint64_t *q_hl_coeffs;
    uint64_t *q_hl_evals;
    uint64_t *q_hr_coeffs;
    uint64_t *q_hr_evals;
    uint64_t *q_h4_coeffs;
    uint64_t *q_h4_evals;
    uint64_t *q_arith_coeffs;
    uint64_t *q_arith_evals;
    uint64_t *range_selector_coeffs;
    uint64_t *range_selector_evals;
    uint64_t *logic_selector_coeffs;
    uint64_t *logic_selector_evals;
    uint64_t *fixed_group_add_selector_coeffs;
    uint64_t *fixed_group_add_selector_evals;
    uint64_t *variable_group_add_selector_coeffs;
    uint64_t *variable_group_add_selector_evals;
    uint64_t *q_lookup_coeffs;
    uint64_t *q_lookup_evals;
    uint64_t *table1;
    uint64_t *table2;
    uint64_t *table3;
    uint64_t *table4;
    uint64_t *left_sigma_coeffs;
    uint64_t *left_sigma_evals;
    uint64_t *right_sigma_coeffs;
    uint64_t *right_sigma_evals;
    uint64_t *out_sigma_coeffs;
    uint64_t *out_sigma_evals;
    uint64_t *fourth_sigma_coeffs;
    uint64_t *fourth_sigma_evals;
    uint64_t *linear_evaluations;
    uint64_t *v_h_coset_8n;
} ProverKeyC;

/* lib.rs:225-229.  powers_of_g: >= D affine points (12 u64 each);
 * powers_of_gamma_g: 2 affine points (unused: hiding is disabled). */
typedef struct {
    const uint64_t *powers_of_g;
    const uint64_t *powers_of_gamma_g;
} CommitKeyC;

/* lib.rs:237-239 / hello.cu:4-6.  Structs by value, ProofC returned by value.
 * Synchronous, device 0.  On any device error it prints and exits, like the
 * reference's CUDA_CHECK (caffe/common.hpp:23-30).  Like the reference
 * (load.cu:311-358) it uploads the prover key and commit key on every call,
 * so a caller may rewrite its key buffers between calls; the folded MSM table
 * of the SRS is kept when the uploaded SRS is byte-identical to the last one.
 * Environment switches (read per call):
 *   PNP_V1_REUSE=1   reuse the keys resident from an earlier call while their
 *                    fingerprint (field pointers, domain, 257 sampled words
 *                    per array) is unchanged: no upload.  Only for callers
 *                    that never mutate key contents in place.
 *   PNP_V1_STRICT=1  exit with PNP_E_ENVELOPE for keys outside the reference
 *                    GPU path's circuit class (non-zero q_m / custom-gate /
 *                    q_lookup selectors or lookup tables): there this backend
 *                    returns the ZK-Garage prover's proof (combine_split,
 *                    widgets, the true z2 shift), which differs byte for byte
 *                    from the reference GPU path's. */
ProofC gen_proof(CircuitC circuit, ProverKeyC pk, CommitKeyC ck);

/* ------------------------------------------------------------------ */
/* 2. v2 ABI — explicit errors, resident keys (additive)               */
/* ------------------------------------------------------------------ */

#define PNP_OK              0
#define PNP_E_ARG          -1   /* bad argument / size                      */
#define PNP_E_DEVICE       -2   /* HIP runtime error                        */
#define PNP_E_NOKEY        -3   /* prover / commit key not loaded           */
#define PNP_E_ENVELOPE     -4   /* key outside the reference GPU path's circuit class
                                       (v1 with PNP_V1_STRICT=1 only) */
#define PNP_E_NOMEM        -5   /* device allocation failed                 */

typedef struct pnp_ctx pnp_ctx;
/* The context the v1 symbol proves on (created by its first call; NULL
 * before).  Its first proof goes without the optional tables (Lagrange basis,
 * copy groups), which then build in the background (v2 pnp_prove likewise on
 * one GPU; PNP_DEFER_TABLES=0 builds them inside the first proof instead,
 * PNP_DEFER_BG=0 inside the second): pnp_sync(pnp_v1_context()) waits for
 * that build, e.g. before timing a steady state.  Extension, diagnostics. */
pnp_ctx *pnp_v1_context(void);

/* Human-readable message of the last error on this thread. */
const char *pnp_last_error(void);

/* One context per GPU; owns the stream, twiddle tables, scratch and keys. */
int pnp_ctx_create(int device, pnp_ctx **out);
void pnp_ctx_destroy(pnp_ctx *ctx);

/* Copy (or adopt) the prover key into HBM once; it stays resident for every
 * later pnp_prove.  domain_size = D (power of two).  If `device_ptrs` is
 * non-zero the pointers are HBM pointers that the context reads in place
 * (they must outlive the context) instead of copying. */
int pnp_load_prover_key(pnp_ctx *ctx, const ProverKeyC *pk, uint64_t domain_size,
                        int device_ptrs);
int pnp_load_commit_key(pnp_ctx *ctx, const CommitKeyC *ck, uint64_t n_points,
                        int device_ptrs);

/* The commit key straight from arkworks' memory, without the per-proof
 * conversion prove_pnp does today (prover.rs:700-711 rebuilds (x, y) tuples
 * of all 2^24+1 SRS points on every call): `points` = the address of
 * commit_key.powers_of_g (Vec<ark_bls12_381::G1Affine>, ark-ec 0.3
 * GroupAffine: x, y Fp384 = 6 u64 Montgomery limbs each (R = 2^384), an
 * `infinity` bool, padding).  The Rust struct's field order is not fixed by
 * the language, so the caller passes the layout it was compiled with:
 * stride = size_of::<G1Affine>() (104 on x86-64), x_off / y_off / inf_off =
 * offset_of!(G1Affine, x / y / infinity).  Only the first n_points points are
 * read (n_points >= the domain size).  A point flagged infinity is refused
 * (PNP_E_ARG: an SRS [tau^i] G never holds it).  device_ptrs: `points` is
 * an HBM address.  Otherwise as pnp_load_commit_key (an unchanged SRS keeps
 * its folded table). */
typedef struct {
    uint64_t stride, x_off, y_off, inf_off;
} pnp_affine_layout;
int pnp_load_commit_key_strided(pnp_ctx *ctx, const void *points, uint64_t n_points,
                                const pnp_affine_layout *layout, int device_ptrs);

/* Which of the 19 commitments of a ProofC (v1 or v2) are the point at
 * infinity: bit k = the k-th CommitmentC of ProofC in declaration order
 * (a_comm 0, b 1, c 2, d 3, z 4, f 5, h_1 6, h_2 7, z_2 8, t_1 .. t_8
 * 9 .. 16, aw_opening 17, saw_opening 18).  Infinity is encoded (x = 0, y = Fq one in Montgomery
 * form), which no curve point has (x = 0 gives y = +-2).  Replaces the
 * hard-coded flags of merkle-tree/src/main.rs:112-123 (f, h1, h2, t7, t8 =
 * true), wrong for any circuit with lookups or a quotient of degree >= 6n. */
#define PNP_PROOF_COMMITMENTS 19
uint32_t pnp_proof_infinity_mask(const ProofC *p);

/* Prove with the resident keys.  `device_ptrs`: the CircuitC witness pointers
 * (q_lookup, w_*) are HBM pointers; pi is always a host pointer. */
int pnp_prove(pnp_ctx *ctx, const CircuitC *cs, int device_ptrs, ProofC *out);

/* pnp_prove with the general public-input set and transcript label of the
 * ZK-Garage prover (Prover::prove_with_preprocessed, prover.rs:171-190: the
 * transcript holds the PublicInputs BTreeMap, pi.rs:16-86), which the v1 ABI
 * cannot carry (CircuitC has one pi / intended_pi_pos, prover.rs:717-725).
 * n_pi pairs (pi_pos[k], pi_canon[4k..4k+4)) — canonical (non-Montgomery)
 * values, host memory, any order; zero values are dropped like
 * PublicInputs::insert; positions must be distinct and < domain size.
 * cs->pi / cs->intended_pi_pos are ignored.  label = NULL is "Merkle tree".
 * With n_pi = 1, a non-zero value and the default label the proof equals
 * pnp_prove's. */
int pnp_prove_ex(pnp_ctx *ctx, const CircuitC *cs, int device_ptrs, uint64_t n_pi,
                 const uint64_t *pi_pos, const uint64_t *pi_canon, const char *label, ProofC *out);

/* Per-stage wall-clock (ms) of the last pnp_prove, for the bench/profiles.
 * Writes up to `cap` doubles and their names; returns the stage count. */
int pnp_last_stage_times(pnp_ctx *ctx, double *ms, const char **names, int cap);

/* Live per-kernel timing with HIP events recorded on the context stream
 * around the named kernels ("msm_accumulate", "quotient"); totals since the
 * last enable.  Used by bench.py for the roofline numbers. */
int pnp_kernel_timing(pnp_ctx *ctx, int enable);
int pnp_kernel_stats(pnp_ctx *ctx, const char *name, double *total_ms, int *launches);
/* Algorithmic bytes the timed launches of `name` were credited with (sum over
 * launches; e.g. msm_accumulate: points*(96 B point + 32 B scalar) of the
 * windows it processed). */
int pnp_kernel_bytes(pnp_ctx *ctx, const char *name, double *bytes);

/* Multi-GPU (one process per GPU, every rank runs pnp_prove on the same
 * inputs and returns the same ProofC).
 *
 * pnp_set_msm_shard: MSMs are sharded by point range — rank r takes points
 * [r*ceil(n/world), ...) over every window (with the folded table of that
 * range) and writes its B partial sums (XYZZ, 192 B each) to
 * d_xbuf + r * bytes_per_rank; after synchronizing its stream the library
 * calls allgather(user, bytes_per_rank), which must leave every rank's slot at
 * its offset in d_xbuf on every rank (an in-place all-gather, e.g. RCCL) and
 * return 0 once the data is visible to the device.  The same exchange carries
 * a few scalars per rank (split polynomial divisions, chunk flags).
 * world = 1 disables.
 *
 * pnp_set_exchange_a2a (optional, before pnp_load_prover_key; world must
 * divide 8): distributes gen_proof's round 4 — rank r owns blocks
 * [r*8/world, (r+1)*8/world) of the 8n coset (residues i mod 8) for the LDEs
 * and the quotient, and coefficient range r of the quotient chunks, the
 * linearisation and the opening witnesses.  One all-to-all moves the inverse
 * block transforms: the library fills world slots of bytes_per_peer at
 * d_a2a (slot s for rank s) and calls alltoall(user, bytes_per_peer), which
 * must leave the slot rank s sent to this rank at
 * d_a2a + (world + s) * bytes_per_peer. */
typedef int (*pnp_allgather_fn)(void *user, uint64_t bytes_per_rank);
/* Every all-gather slot ends with one tag word naming the exchange (the last
 * 8 bytes of each rank's bytes_per_rank): an exchange harness can tell the
 * messages apart without inferring them from sizes, and the library refuses
 * (PNP_E_DEVICE, "out of step") a result in which a peer's tag differs. */
#define PNP_EX_TAG_COUNTS    0xB0C4E7C0ULL  /* bucket-range MSMs: entry bytes per destination */
#define PNP_EX_TAG_MSM_SUMS  0x5EC7A111ULL  /* point-range MSMs: B partial sums (XYZZ)       */
#define PNP_EX_TAG_T_FLAGS   0x7F1A6500ULL  /* round 4: non-zero quotient chunks (8 words)   */
#define PNP_EX_TAG_DIV_CARRY 0xD1FC0001ULL  /* split divisions by (X - z): slice values   */
#define PNP_EX_TAG_EVALS     0xE7A15000ULL  /* round 5: partial evaluations (18 x 4 words)  */
#define PNP_EX_TAG_STATUS    0x57A7A500ULL  /* key load / derived tables: per-rank status   */
#define PNP_EX_TAG_DEVICE    0xDE71CE00ULL  /* key load: which GPU each rank runs on        */
typedef int (*pnp_alltoall_fn)(void *user, uint64_t bytes_per_peer);
/* pnp_set_exchange_v (optional, before the first commitment; world must
 * divide the bucket count): the folded MSMs shard BUCKET ranges instead of
 * point ranges — rank s owns buckets [s NB/world, (s+1) NB/world) of every MSM
 * of a batch, so each rank sorts, accumulates and reduces 1/world of the
 * buckets (the point-range scheme reduces all of them on every rank).  Each
 * rank digitises its own point range and sends every entry (8 bytes) to its
 * bucket's owner: the library writes world segments to d_send (segment s,
 * send_bytes[s] bytes, for rank s, back to back in rank order) and calls
 * alltoallv(user, send_bytes, recv_bytes), which must leave the segment rank s
 * sent to this rank at offset recv_bytes[0] + ... + recv_bytes[s-1] of d_recv
 * (recv_bytes comes from a preceding all-gather of the counts).  A batch whose
 * segments would not fit `capacity_bytes` (pathological scalars that crowd one
 * bucket range) falls back to point ranges.  The commit key's folded table then
 * covers all n points on every rank (6.5 GiB at n = 2^22). */
typedef int (*pnp_alltoallv_fn)(void *user, const uint64_t *send_bytes, const uint64_t *recv_bytes);
/* The library's HIP stream (a hipStream_t): every kernel and copy of a proof
 * runs on it in order.  An exchange that enqueues its collectives on this
 * stream (RCCL: libpnp_rccl.so, include/pnp_rccl.h) declares itself with
 * pnp_set_exchange_ordered(ctx, 1): the library then calls the callbacks
 * without synchronising the stream first, and a callback returns once its
 * collective is enqueued (the library's next copies and kernels are ordered
 * behind it).  Default 0: the stream is synchronised before every callback,
 * which must return with the data visible to the device (host-memory
 * exchanges, other streams). */
int pnp_ctx_stream(pnp_ctx *ctx, void **stream);
int pnp_set_exchange_ordered(pnp_ctx *ctx, int ordered);
int pnp_set_msm_shard(pnp_ctx *ctx, int rank, int world, pnp_allgather_fn allgather,
                      void *user, uint64_t *d_xbuf, uint64_t xbuf_bytes);
int pnp_set_exchange_a2a(pnp_ctx *ctx, pnp_alltoall_fn alltoall, void *user, uint64_t *d_a2a,
                         uint64_t a2a_bytes);
int pnp_set_exchange_v(pnp_ctx *ctx, pnp_alltoallv_fn alltoallv, void *user, uint64_t *d_send,
                       uint64_t *d_recv, uint64_t capacity_bytes);

/* ------------------------------------------------------------------ */
/* 3. Operator API on HBM pointers (mirrors PLONK/utils/function.cuh) */
/*    All ops are asynchronous on the context stream; pnp_sync waits.  */
/* ------------------------------------------------------------------ */

int pnp_sync(pnp_ctx *ctx);

/* In-place natural-order radix-2 NTT of 2^lg_n Montgomery Fr
 * (function.cu:249-273 Ntt / Intt; arkworks fft / ifft semantics).
 * inverse=1 multiplies by n^-1.  coset=1 applies the g=7 coset
 * (forward: x_i *= g^i before, inverse: x_i *= g^-i after). */
int pnp_ntt(pnp_ctx *ctx, uint64_t *d_inout, uint32_t lg_n, int inverse, int coset);

/* Ntt_coset::forward (function.cu:261-267): zero-pad n -> 8n, coset NTT. */
int pnp_coset_lde8(pnp_ctx *ctx, const uint64_t *d_coeffs, uint64_t *d_out8, uint32_t lg_n);

/* commit (KZG/kzg10.cu:31-44): MSM of n affine points with n Montgomery
 * scalars (converted to canonical inside, arithmetic.cu:3-8), result as
 * affine Montgomery point (infinity -> x=0, y=Fq one). Synchronous. */
int pnp_commit(pnp_ctx *ctx, const uint64_t *d_points, const uint64_t *d_scalars,
               uint64_t n, CommitmentC *out);

/* KZG commit (kzg10.cu:31-55) against the RESIDENT commit key
 * (pnp_load_commit_key): sum_{i<n} s_i powers_of_g[i], as gen_proof's
 * commitments.  Uses the folded fixed-base layout (2^(c k) multiples of the
 * first n SRS points, built on the first call for this n and kept).  */
int pnp_commit_ck(pnp_ctx *ctx, const uint64_t *d_scalars, uint64_t n, CommitmentC *out);

/* Extension (no reference counterpart; what gen_proof's round 1 uses): the
 * KZG commitment of the polynomial given by its n evaluations on the order-n
 * subgroup <omega> (natural order, Montgomery) — the same point as
 * pnp_commit_ck over its coefficients iNTT(evals), computed as
 * sum_i evals_i [L_i(tau)] G against the resident commit key in the Lagrange
 * basis (derived from the first n SRS points on the first call for this n and
 * kept; zero evaluations cost nothing).  n a power of two <= the key's points.
 * PNP_E_ARG when the basis is unavailable (PNP_LAGRANGE=0, degenerate key).  */
int pnp_commit_evals(pnp_ctx *ctx, const uint64_t *d_evals, uint64_t n, CommitmentC *out);

/* HBM accounting (extension): out[0] = device bytes this library holds now
 * (every context of the process), out[1] = their peak since the previous
 * pnp_hbm_usage call (which restarts it), and for the loaded
 * prover key the upper bounds pnp_load_prover_key budgets a proof with, still
 * to be allocated on this rank: out[2] mandatory (per-proof buffers, NTT
 * tables, the commit key's folded table, MSM work), out[3] the Lagrange-basis
 * key + table, out[4] the copy-constraint groups + table, out[5] the largest
 * build scratch.  The first pnp_prove after a key load checks them against
 * the rank's share of its GPU's free HBM: it fails with PNP_E_NOMEM before any
 * work (every rank of a multi-GPU run, naming the short one) when out[2] +
 * out[5] does not fit, and switches the optional tables off (same proof bytes)
 * when they do not. */
int pnp_hbm_usage(pnp_ctx *ctx, uint64_t out[6]);

/* Extension (operator form of gen_proof's copy-group commitments, wires.hip):
 * B <= 16 MSMs over sub-ranges of ONE base set — out[b] = sum_{i<n}
 * s_b[i] P[seg_off[b] + i] over the n_points affine points d_points (12 u64
 * each, Montgomery) — through one folded table built over all n_points (the
 * segmented batch of the round-1 wire commitments; each MSM's entries carry its
 * segment offset).  seg_off[b] + n <= n_points.  Single GPU.  Synchronous.  */
int pnp_commit_segments(pnp_ctx *ctx, const uint64_t *d_points, uint64_t n_points, int B,
                        const uint64_t *seg_off, const uint64_t *const *d_scalars, uint64_t n,
                        CommitmentC *out);

/* evaluate (function.cu:162-173): sum_i c_i x^i; x and result Montgomery,
 * host-side scalars.  Synchronous. */
int pnp_poly_eval(pnp_ctx *ctx, const uint64_t *d_coeffs, uint64_t n,
                  const uint64_t x[4], uint64_t out[4]);

/* poly_div_poly with c = -z (kzg10.cu:87-99): in place, p <- p / (X - z),
 * remainder dropped, top coefficient set to zero. */
int pnp_poly_div_linear(pnp_ctx *ctx, uint64_t *d_poly, uint64_t n, const uint64_t z[4]);

/* accumulate_mul_poly (mont_arithmetic.cu:334-360): out[0]=1,
 * out[i] = prod_{j<i} in[j]; in place. */
int pnp_prefix_product(pnp_ctx *ctx, uint64_t *d_inout, uint64_t n);

/* Batch inverse in place (inv(0) = 0, like the reference inv_mod kernel). */
int pnp_batch_inverse(pnp_ctx *ctx, uint64_t *d_inout, uint64_t n);

/* ------------------------------------------------------------------ */
/* 4. Synthetic-input utilities (bench / test plumbing, not the path)  */
/* ------------------------------------------------------------------ */

/* d_out[i] = uniform-ish Montgomery Fr from a counter-based hash of (seed,i). */
int pnp_synth_random_fr(pnp_ctx *ctx, uint64_t *d_out, uint64_t n, uint64_t seed);
/* d_out[i] = tau^i * G1 generator, affine Montgomery (an SRS); tau Montgomery. */
int pnp_synth_srs(pnp_ctx *ctx, uint64_t *d_out, uint64_t n, const uint64_t tau[4]);
/* Satisfying random arithmetic circuit on the n-domain (tests/bench):
 * in:  w[0] = a, w[3] = d (n_gates each), sel[0..7] = q_l q_r q_o q_4 q_c q_hl
 *      q_hr q_h4 evaluations (n each, rows >= n_gates ignored);
 * out: w[1] = b (b_i = a_pi(i)), w[2] = c (solved from the gate), sel[8] =
 *      q_arith evaluations, sigma[0..3] evaluations (copy cycles b_i <-> a_pi(i)). */
int pnp_synth_circuit(pnp_ctx *ctx, uint64_t *const w[4], uint64_t *const sel[9],
                      uint64_t *const sigma[4], uint64_t n, uint64_t n_gates, uint64_t pi_pos,
                      const uint64_t pi_canon[4]);
/* The reference's own Poseidon Merkle-tree circuit of height `height`
 * (merkle-tree/src/constraints.rs:20-107 laid out like the reference composer;
 * 193 (2^(height-1) - 1) + 5 gates, mirrors tests/merkle_circuit.py):
 * in:  consts = 199 canonical Fr (4 limbs each): the 189 Poseidon round
 *      constants, the 3x3 MDS matrix row-major, the domain tag;
 *      d_leaves = 2^(height-1) Montgomery Fr, d_blind = 8 Montgomery Fr (the
 *      two blinding rows of StandardComposer::new);
 * out: d_nodes = the 2^(height-1) - 1 tree nodes (level order, root first),
 *      w[0..3] wire values of the gates, sel[0..8] = q_l q_r q_o q_4 q_c q_hl
 *      q_hr q_h4 q_arith and sigma[0..3] evaluations on the n-domain,
 *      root_canon = the root (PI = -root at row gates - 1). */
int pnp_synth_merkle(pnp_ctx *ctx, uint32_t height, const uint64_t *consts, const uint64_t *d_leaves,
                     const uint64_t *d_blind, uint64_t *d_nodes, uint64_t *const w[4], uint64_t *const sel[9],
                     uint64_t *const sigma[4], uint64_t n, uint64_t root_canon[4]);
/* d_out[i] = (g * w_8n^i)^n - 1 (v_h on the 8n coset) and the coset points. */
int pnp_synth_coset_consts(pnp_ctx *ctx, uint64_t *d_vh, uint64_t *d_x, uint32_t lg_n);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#ifdef __cplusplus
static_assert(sizeof(CommitmentC) == 96, "CommitmentC layout (lib.rs:231-235)");
static_assert(sizeof(ProofEvaluationsC) == 26 * 32, "ProofEvaluationsC layout");
static_assert(sizeof(ProofC) == 2656, "ProofC layout (lib.rs:120-142)");
static_assert(sizeof(CircuitC) == 72, "CircuitC layout (lib.rs:144-155)");
static_assert(sizeof(ProverKeyC) == 44 * 8, "ProverKeyC layout (lib.rs:157-223)");
static_assert(sizeof(CommitKeyC) == 16, "CommitKeyC layout (lib.rs:225-229)");
#else
_Static_assert(sizeof(ProofC) == 2656, "ProofC layout (lib.rs:120-142)");
_Static_assert(sizeof(ProverKeyC) == 44 * 8, "ProverKeyC layout (lib.rs:157-223)");
#endif

#endif /* PNP_PLONK_H */
