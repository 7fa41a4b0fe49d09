// context.h — the per-GPU context behind the C-ABI (replaces the reference's
// per-op SyncedMemory allocation, lib/caffe/syncedmem.cpp): one stream, the
// NTT tables, MSM work buffers, a scratch pool and the HBM-resident keys.
#pragma once
#include "pnp_internal.h"
#include <array>
#include <atomic>
#include <memory>
#include <thread>

struct pnp_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // low-priority side stream for challenge-independent work overlapped with
    // the MSMs (prover.cpp), created on first use, and its events
    hipStream_t stream_lo = nullptr;
    hipEvent_t ev_fork = nullptr, ev_w8 = nullptr, ev_z8 = nullptr;
    hipStream_t side_stream();
    pnp::NttTables ntt;
    pnp::MsmWork msm;
    pnp::DevBuf scratch_a, scratch_b;
    // pinned staging of the host -> HBM uploads (abi.cpp h2d_batch): per copy
    // thread two chunks, a stream and an event per chunk; made on first use
    static constexpr int kStgThreads = 6;
    void *stg_buf[2 * kStgThreads] = {};
    hipStream_t stg_st[kStgThreads] = {};
    hipEvent_t stg_ev[2 * kStgThreads] = {};

    // ---- resident prover key (ProverKeyC mirrored in HBM) ----
    bool pk_loaded = false;
    uint64_t pk_n = 0;                     // domain size D
    std::vector<pnp::DevBuf> pk_owned;     // copies (device_ptrs == 0), by ProverKeyC field
    ProverKeyC pk_dev{};                   // HBM pointers for every field
    bool pk_qm_zero = false, pk_qlookup_zero = false;  // all-zero 8n selector evaluations
    bool pk_custom_nz[4] = {};  // range, logic, fixed-base, curve-add selectors non-zero
    pnp::DevBuf pk_sigma_n[4];             // sigma evaluations on the n-domain
    pnp::DevBuf pk_tmp[4];                 // key-load scratch (8n Fr each), kept for the next load
    // The quotient's 8n-point arrays in block layout (ntt.hip: point 8j + m
    // -> block m, index j), blocks pk_mb0 .. pk_mb0 + pk_nb - 1 only:
    // q_* selectors, sig0..3, lin (coset points) and the proof-independent
    // coset constants computed at key load: vh_inv = v_h^-1 and, when
    // pk_std_coset (linear_evaluations = 7 w_8n^i, v_h = x^n - 1),
    // l1v = n^-1 / (x - 1) = L1 / Z_H
    std::map<std::string, pnp::DevBuf> pk_blk;
    int pk_mb0 = 0, pk_nb = 8, pk_blk_rank = 0, pk_blk_world = 1;
    bool pk_std_coset = false;
    pnp::DevBuf pk_pinv;                   // 1 / (x - w^pos) (block layout), pos = pk_pinv_pos
    uint64_t pk_pinv_pos = ~0ULL;
    const uint64_t *blk(const char *name) const {
        auto it = pk_blk.find(name);
        return it == pk_blk.end() ? nullptr : it->second.u64();
    }
    // the same block arrays in the 2^261 form for k_quotient29 (protocol.h),
    // made at key load for keys of its class (pk_q29): selectors, sigmas, lin
    std::map<std::string, pnp::DevBuf> pk_blk29;
    bool pk_q29 = false;
    const uint64_t *blk29(const char *name) const {
        auto it = pk_blk29.find(name);
        return it == pk_blk29.end() ? nullptr : it->second.u64();
    }
    // ---- resident commit key ----
    bool ck_loaded = false;
    uint64_t ck_points = 0;
    pnp::DevBuf ck_owned;
    const uint64_t *ck_dev = nullptr;
    // device-pointer loads: the content hash of the SRS the derived tables
    // (folded tables, Lagrange basis, groups) were built from — a reload of
    // the same bytes keeps them
    uint64_t ck_hash[2] = {0, 0};
    bool ck_hash_valid = false;
    // folded MSM table of the first ck_table_n SRS points (msm_build_table),
    // built on the first commitment of that size
    pnp::DevBuf ck_table;
    uint64_t ck_table_n = 0, ck_table_p0 = 0, ck_table_p1 = 0;
    // the first lag_n SRS points in the Lagrange basis of the order-lag_n
    // subgroup (srs_lagrange, affine) and their folded table: witness
    // polynomials are committed from their evaluations (lagrange.hip); built
    // on the first commitment of that size; lag_ok = false: degenerate key
    pnp::DevBuf lag_points, lag_table;
    uint64_t lag_n = 0, lag_table_n = 0, lag_table_p0 = 0, lag_table_p1 = 0;
    bool lag_ok = false;
    // wire commitments over copy-constraint groups (wires.hip): the rows of
    // one wire that hold one variable (a cycle of sigma restricted to the
    // wire) share the base sum_i L_i, so a wire commits with one scalar per
    // group; built from sigma and the Lagrange points on the first proof that
    // needs them, kept while both are unchanged
    // Index 4 is z (round 3): its groups are the runs of rows sigma fixes
    // (the padding rows: z is constant there).
    struct WireBases {
        bool built = false, ok = false, wires_ok = false, z_ok = false;
        bool sliced = false;            // the table holds this rank's point range of each segment
        int c = 0;                      // its window bits (msm_fold_c of one segment's n)
        uint64_t n = 0, total = 0, m = 0, len = 0;  // domain, bases, largest group count, MSM length
        uint64_t g[5] = {}, off[5] = {};
        bool ident[5] = {};             // ungrouped wire: its scalars are its evaluations
        pnp::DevBuf grp[5], rep[5];     // row -> group slot, slot -> representative row
        pnp::DevBuf scal[5];            // per-proof group scalars at their slots (n each)
        pnp::DevBuf table;              // folded table over the `total` bases
        pnp::DevBuf sigma;              // the sigma evaluations the groups came from
        pnp::DevBuf flag;
        uint64_t pk_gen = 0;            // prover-key load the sigma check last covered
    } wb;
    uint64_t pk_gen = 0;                // incremented by every pnp_load_prover_key
    // the key-load HBM budget (pnp_load_prover_key) left no room for these
    // optional tables: the prover commits without them (same proof bytes)
    // (atomic: the background builder's failure paths set them while a proof
    // on the owning thread may read them; such a proof finds the build busy and
    // commits without the tables whatever it reads)
    std::atomic<bool> hbm_lag_off{false}, hbm_groups_off{false};
    bool hbm_checked = false;  // the budget of the loaded keys has been checked (first proof)
    // Deferred tables: the context's first proof commits without the
    // optional tables it would have to build first (Lagrange basis, copy
    // groups: ~3.4 s at 2^22), so a caller that proves once per process pays
    // its upload and proof only; same proof bytes either way.  On one GPU the
    // tables are then built in the background (bg_*: a thread on a
    // lowest-priority stream, one kernel in flight at a time) while the caller
    // goes on, and the first proof after the build finished uses them; with
    // several ranks the next proof builds them (the builds exchange status
    // with the peers).  PNP_DEFER_TABLES=1 / 0 forces it on / off; default:
    // on at world 1.  Once per context, so a caller reloading its keys every
    // call (PNP_V1_RELOAD) still gets the tables from then on
    int defer_tables = -1;   // -1: the default for the world size (resolved by the first proof)
    bool defer_now = false;  // this proof defers (set per proof)
    bool tables_wanted = false;  // this deferring proof found a table missing
    uint64_t proofs_started = 0;
    std::thread bg;
    std::atomic<int> bg_state{0};  // 0 idle, 1 building, 2 finished (not yet joined)
    std::atomic<bool> bg_cancel{false};
    hipStream_t bg_stream = nullptr;

    // ---- per-proof working set (sized on first use, reused) ----
    std::map<std::string, pnp::DevBuf> work;
    uint64_t *buf(const std::string &name, size_t elems_fr);

    pnp::KernelTimer ktimer;

    // ---- stage timing of the last proof ----
    std::vector<std::pair<std::string, double>> stages;
};

namespace pnp {
// bytes a proof at domain n still has to allocate on this rank (abi.cpp)
struct HbmPlan {
    uint64_t mandatory = 0;  // per-proof buffers, NTT tables, commit-key table, MSM work
    uint64_t lag = 0;        // the Lagrange-basis key and its folded table (optional)
    uint64_t groups = 0;     // the copy-constraint groups and their table (optional)
    uint64_t transient = 0;  // the largest build scratch on top of them (max of the three below)
    uint64_t t_mand = 0, t_lag = 0, t_groups = 0;  // build scratch of the commit-key table, Lagrange, groups
};
HbmPlan hbm_plan(pnp_ctx *ctx, uint64_t n);
// multi-GPU: AND of every rank's `mine` (one tagged all-gather); world 1: mine
bool all_ranks_ok(pnp_ctx *ctx, bool mine);
bool lagrange_enabled();
// the HBM budget of the loaded keys, checked by the first proof (sets
// hbm_lag_off / hbm_groups_off, or throws PNP_E_NOMEM)
void hbm_budget(pnp_ctx *ctx);
bool wire_groups_enabled();
Fr root_of_unity(uint32_t lg);
Fr fr_from_u64(uint64_t x);
// drop everything derived from the resident SRS (folded tables, Lagrange basis)
void ck_derived_reset(pnp_ctx *ctx);
// commitments over the resident SRS (folded MSM)
const uint64_t *commit_table(pnp_ctx *ctx, uint64_t n);
// host -> HBM copies of caller buffers (pageable memory) through pinned
// staging chunks, several copy threads at once; returns when they have landed
struct H2D {
    void *dst;
    const void *src;
    size_t bytes;
};
void h2d_batch(pnp_ctx *ctx, const std::vector<H2D> &copies);
// the folded table of the Lagrange-basis SRS of size n (this rank's point
// range), nullptr when it is unavailable (PNP_LAGRANGE=0, n not a power of
// two or above the key, degenerate key)
const uint64_t *lagrange_table(pnp_ctx *ctx, uint64_t n);
// B commitments of polynomials given by their n evaluations on the order-n
// subgroup (Montgomery Fr, natural order): sum_i e_i L_i; requires
// lagrange_table(ctx, n) != nullptr
void commit_evals_batch(pnp_ctx *ctx, const uint64_t *const *d_evals, int B, uint64_t n, CommitmentC *const *out);
void commit_affine(pnp_ctx *ctx, const uint64_t *d_scalars, uint64_t n, CommitmentC *out);
// the four wire commitments from their n padded evaluations over the
// copy-constraint-grouped bases (wires.hip); false (nothing written) when the
// groups are unavailable or the witness differs inside a group, and the caller
// commits with commit_evals_batch
bool commit_wires_grouped(pnp_ctx *ctx, const uint64_t *const *d_evals, uint64_t n, CommitmentC *const *out);
// z (round 3) from its n evaluations over its groups, the runs of rows sigma
// fixes (wires.hip); false when unavailable (the caller commits row by row)
bool commit_z_grouped(pnp_ctx *ctx, const uint64_t *d_z, uint64_t n, CommitmentC *out);
// drop the wire groups (a new commit key or Lagrange basis)
void wire_bases_reset(pnp_ctx *ctx);
// build the copy-constraint groups now if they are enabled and missing
// (wires.hip; the background table build)
void wire_bases_build(pnp_ctx *ctx, uint64_t n);
// ---- the background table build (abi.cpp; see pnp_ctx::bg) ----
// start it after a deferring proof (world 1)
void tables_start_background(pnp_ctx *ctx, uint64_t n);
// PNP_DEFER_BG (default on): world-1 deferral builds in the background
bool tables_bg_enabled();
// true while it runs (joins it once it has finished); a proof then goes
// without the tables.  Always false on the builder's own thread
bool tables_busy(pnp_ctx *ctx);
// wait for it (pnp_sync, key loads, operator calls that need the tables)
void tables_wait(pnp_ctx *ctx);
// stop it at its next kernel and wait (context destruction, process exit)
void tables_cancel(pnp_ctx *ctx);
// the stream the table builds run on: the background stream on the builder's
// thread, else the context stream
hipStream_t tables_stream(pnp_ctx *ctx);
// B commitments over the resident SRS in one batched MSM
// local: on a multi-GPU run the scalars hold only this rank's point range
void commit_affine_batch(pnp_ctx *ctx, const uint64_t *const *d_scalars, int B, uint64_t n,
                         CommitmentC *const *out, bool local = false);
// v2 options of pnp_prove_ex: public inputs (positions, canonical values) and
// the transcript label; nullptr = the v1 contract (one PI from the circuit,
// label "Merkle tree")
struct ProveOpts {
    uint64_t n_pi;
    const uint64_t *pi_pos, *pi_canon;
    const char *label;
};
int prove_impl(pnp_ctx *ctx, const CircuitC *cs, int device_ptrs, ProofC *out, const ProveOpts *opt = nullptr);
}  // namespace pnp
