// pnp_internal.h — host-side declarations shared by the HIP translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <map>
#include <string>
#include <tuple>
#include <vector>
#include "field.cuh"
#include "../../include/pnp_plonk.h"

namespace pnp {

void set_error(const char *fmt, ...);

#define PNP_HIP(expr)                                                              \
    do {                                                                           \
        hipError_t e_ = (expr);                                                    \
        if (e_ != hipSuccess) {                                                    \
            ::pnp::set_error("%s:%d %s: %s", __FILE__, __LINE__, #expr,            \
                             hipGetErrorString(e_));                               \
            throw ::pnp::Error(PNP_E_DEVICE);                                      \
        }                                                                          \
    } while (0)

struct Error {
    int code;
    explicit Error(int c) : code(c) {}
};

// device buffer with RAII
struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    explicit DevBuf(size_t b) { alloc(b); }
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    DevBuf(DevBuf &&o) noexcept : p(o.p), bytes(o.bytes) { o.p = nullptr; o.bytes = 0; }
    DevBuf &operator=(DevBuf &&o) noexcept {
        if (this != &o) { release(); p = o.p; bytes = o.bytes; o.p = nullptr; o.bytes = 0; }
        return *this;
    }
    ~DevBuf() { release(); }
    void alloc(size_t b);
    void release();
    uint64_t *u64() const { return static_cast<uint64_t *>(p); }
};

// ---- NTT (ntt.hip) ----
struct NttTables {
    // tw[e] = w_N^e, e < N/2, for forward and inverse roots, per lg
    std::map<uint32_t, DevBuf> fwd, inv;
    // the same twiddles as dense rows per shift (ntt.hip ntt_twiddle_rows): row
    // sh = w_N^(i 2^sh), i < N / 2^(sh+1), at offset N - N / 2^sh
    std::map<uint32_t, DevBuf> fwd_rows, inv_rows;
    DevBuf coset_hi, coset_lo;        // g^(4096 k), g^k
    DevBuf coset_inv_hi, coset_inv_lo;  // g^-(4096 k), g^-k
    bool coset_ready = false;
    // coset LDE twist per lg_n: (g w_8n^rev3(b))^j for block b, j < n
    std::map<uint32_t, DevBuf> lde_twist;
    // block layout twists per lg_n: (g w_8n^m)^j and w_8n^(-m j), block m
    std::map<uint32_t, DevBuf> blk_twist, blk_twist_inv;
    // the same twiddles / twists times 2^261 in radix 2^29 (9 u32 per entry)
    // for the radix-2^29 passes (fr29.cuh)
    std::map<uint32_t, DevBuf> fwd29, inv29, blk_twist29, blk_twist_inv29;
    // the forward block twists times 32 (lde_blocks form29), and their 2^261 form
    std::map<uint32_t, DevBuf> blk_twist32, blk_twist32_29;
};
const uint64_t *ntt_twiddles(NttTables &t, uint32_t lg, bool inverse, hipStream_t s);
void ntt_prepare_coset(NttTables &t, hipStream_t s);
// natural-order NTT of 2^lg elements in place, or from `src` into d (the first
// pass reads src: no separate copy)
void ntt_run(NttTables &t, uint64_t *d, uint32_t lg, bool inverse, bool coset, hipStream_t s,
             const uint64_t *src = nullptr);
// out8[i] = i < n ? in[i] * g^i : 0, then forward NTT of size 8n (Ntt_coset::forward)
void coset_lde8(NttTables &t, const uint64_t *in, uint64_t *out8, uint32_t lg_n, hipStream_t s);

// block layout of the 8n coset (point i = 8 j + m -> block m, index j):
// LDE of n coefficients into blocks m0 .. m0+nb-1 (any nb, m0 + nb <= 8)
// build every NTT table of domain 2^lg_n on stream s (before forking work
// that reads them onto another stream)
void ntt_warm(NttTables &t, uint32_t lg_n, hipStream_t s);
// form29: the values times 32, i.e. in the 2^261 form of fr29.cuh (k_quotient29)
void lde_blocks(NttTables &t, const uint64_t *in, uint64_t *out, uint32_t lg_n, int m0, int nb,
                hipStream_t s, bool form29 = false);
// per block: unscaled inverse size-n DFT then twist by w_8n^(-m u)
void intt_blocks(NttTables &t, uint64_t *d, uint32_t lg_n, int m0, int nb, hipStream_t s);
// 8-point inverse DFT across blocks + g^-i / (8n): coefficient chunks u in [q0, q0+len)
void t_combine(NttTables &t, const uint64_t *Y, uint64_t len, uint64_t q0, uint64_t *out,
               uint32_t lg_n, unsigned *nz, hipStream_t s);
// coefficient chunks t_1 .. t_nb (out[k n + u]) from blocks 0 .. nb-1 after
// intt_blocks, for deg t < nb n (nb = 6 .. 8; 8 is t_combine).  Both OR into
// the device word *nz bit k when chunk k has a non-zero coefficient.
void t_combine_blocks(NttTables &t, const uint64_t *Y, int nb, uint64_t *out, uint32_t lg_n, unsigned *nz,
                      hipStream_t s);
void to_blocks(const uint64_t *in, uint64_t *out, uint32_t lg_n, int m0, int nb, hipStream_t s);

// ---- live per-kernel timing with HIP events on the launching stream ----
struct KernelTimer {
    bool enabled = false;
    struct Stat {
        double ms = 0, bytes = 0;
        int launches = 0;
    };
    struct Pending {
        std::string name;
        hipEvent_t e0, e1;
        double bytes;
    };
    std::map<std::string, Stat> stats;
    std::vector<Pending> pending;
    std::vector<hipEvent_t> pool;
    hipEvent_t get();
    void begin(const char *name, hipStream_t s, hipEvent_t &e0);
    // `bytes`: algorithmic bytes credited to this launch
    void end(const char *name, hipStream_t s, hipEvent_t e0, double bytes = 0);
    void collect();  // call after the stream is synchronized
    // add `units` to a counter read back with pnp_kernel_bytes (no timing)
    void credit(const char *name, double units) {
        if (enabled) stats[name].bytes += units;
    }
};

// Background table builds (abi.cpp tables_start_background): on the builder's
// thread every build kernel is followed by bg_step, which waits for it (one
// build kernel in flight at a time, so a proof's streams never queue behind
// more than one of them on a shared hardware queue) and stops the build when
// it is cancelled.  A no-op on every other thread.
extern thread_local bool t_bg_build;
void bg_step(hipStream_t s);

// ---- MSM (msm.hip) ----
// buffers of one group of an MSM batch: counts (coarse-bin counts -> offsets,
// scan_tmp), ent/fkey (pass-A entries and fine keys), offsets (bucket
// starts), sorted (entries by bucket), buckets (XYZZ buckets + reduction tree),
// seg (split-bucket pieces), redo (segments the radix-2^29 accumulation hands
// back to the exact path)
struct MsmGroup {
    DevBuf counts, offsets, scan_tmp, ent, fkey, sorted, buckets, seg, redo;
    DevBuf exc;  // folded: an F29 merge / tree addition met equal or opposite operands
    DevBuf heavy;  // folded: the merge's queue of buckets with many pieces
    uint32_t S = 0, pieces = 0;  // folded: accumulate segment length, pieces per bucket
    uint64_t nthr = 0;           // folded: accumulate lanes (head / tail slots)
    // timed runs only (KernelTimer enabled): what the last k_accumulate29 launch
    // really did, counted on the device from the bucket starts — {sorted
    // entries, pieces started fresh}; mixed additions = entries - pieces
    DevBuf wctr;
    unsigned long long wctr_h[65] = {};  // entries, then 64 piece counters (msm.hip k_count_pieces)
    bool wctr_live = false;
};
struct MsmWork {
    DevBuf digits;  // u32 keys of every (MSM, window, point)
    MsmGroup grp[2];  // the two pipelined groups of a batch
    hipStream_t s2 = nullptr;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    KernelTimer *timer = nullptr;
    // point-range sharding across ranks (pnp_set_msm_shard)
    // window bits of the folded layout (msm_cfg default when 0; PNP_FOLD_C)
    int fold_c = 0;
    int rank = 0, world = 1;
    pnp_allgather_fn allgather = nullptr;
    void *user = nullptr;
    uint64_t *xbuf = nullptr;
    uint64_t xbuf_bytes = 0;
    // all-to-all for the distributed quotient (pnp_set_exchange_a2a)
    pnp_alltoall_fn alltoall = nullptr;
    void *a2a_user = nullptr;
    uint64_t *a2a = nullptr;
    uint64_t a2a_bytes = 0;
    // variable all-to-all of the bucket-range sharded MSMs (pnp_set_exchange_v):
    // rank s owns buckets [s NB/W, (s+1) NB/W) of every MSM, the entries travel
    // to their bucket's owner; unset: point-range sharding
    pnp_alltoallv_fn alltoallv = nullptr;
    void *v_user = nullptr;
    uint64_t *v_send = nullptr, *v_recv = nullptr;
    uint64_t v_bytes = 0;
    // the exchange callbacks enqueue their collectives on the library's
    // stream (pnp_set_exchange_ordered: RCCL on pnp_ctx_stream): the data they
    // move is ordered behind the work that made it, no host synchronisation
    // before a callback; otherwise (host-memory exchanges) the stream is
    // synchronised first
    bool ordered = false;
    // the folded table covers ALL n points (bucket ranges gather any point)
    bool full_table() const { return world > 1 && alltoallv != nullptr; }
    DevBuf part_counts, rec_counts;  // bucket-range pass counts
    // Fixed-slot bucket exchange (msm.hip msm_bucket_batch): every rank sends
    // every peer one slot of `cap` records with the bin counts in the slot's
    // header, so the records move in one equal-size all-to-all with no host
    // round trip to size it.  cap is per batch of a proof (its ordinal since
    // the proof began, B, the table's n), set from the all-gathered counts of
    // that batch's first variable-size run (the same on every rank); a batch
    // whose counts outgrow it is redone on the variable path, which raises it.
    // PNP_MSM_SLOTS=0: always the variable path.
    std::map<std::tuple<uint32_t, int, uint64_t>, uint64_t> slot_cap;
    uint32_t batch_seq = 0;  // bucket-range batches since the proof began
    DevBuf slot_dev;         // run table, bin starts, flags, per-destination counts
    unsigned long long slot_runs = 0, slot_overflows = 0;  // slotted batches / redone ones
};
// before an exchange callback: the data on the stream is complete
inline void ex_fence(const MsmWork &wk, hipStream_t s) {
    if (!wk.ordered) PNP_HIP(hipStreamSynchronize(s));
}
// all-gather of k words per rank (rank-major result, world x k), every slot
// tagged (PNP_EX_TAG_*, include/pnp_plonk.h) and the tags checked
std::vector<uint64_t> rank_allgather(MsmWork &wk, hipStream_t s, const uint64_t *mine, int k, uint64_t tag);
// sum_i s_i P_i; scalars Montgomery Fr; result written to host as XYZZ Fq (4x6 u64)
// `table` (optional): msm_build_table(d_points, n) — the folded layout
void msm_run(MsmWork &w, const uint64_t *d_points, const uint64_t *d_scalars_mont, uint64_t n,
             uint64_t *h_xyzz, hipStream_t s, const uint64_t *table = nullptr);
// A folded table built over n_table points holding several point sets: MSM b
// of a batch sums over points off[b] .. off[b] + n - 1 of it (wires.hip: the
// four wires' grouped bases in one table)
struct MsmSegs {
    uint64_t n_table = 0;
    uint64_t off[16] = {};
    // multi-GPU point ranges: the table holds only this rank's slice [p0, p1)
    // of every set (msm_point_range of the MSM length), off[] are the slices'
    // starts in it — 1/world of the full table
    bool sliced = false;
    // window bits of the table (0: msm_cfg(n_table)); a table over several
    // point sets takes the width for ONE set's size (msm_fold_c(n)): its
    // buckets serve one set per MSM
    int c = 0;
};
// the folded layout's window bits for an MSM over n_points points
int msm_fold_c(uint64_t n_points, int fold_c);
// scalars_local: multi-GPU, d_scalars[b] hold only this rank's point range
// segs: `table` is segmented as above (d_points unused)
void msm_run_batch(MsmWork &w, const uint64_t *d_points, const uint64_t *const *d_scalars, int B,
                   uint64_t n, uint64_t *h_xyzz, hipStream_t s, const uint64_t *table = nullptr,
                   bool scalars_local = false, const MsmSegs *segs = nullptr);
// HBM of the MSM machinery, upper bounds (the key-load budget): a folded table
// over n_points (windows of a table for n_cfg points), its build scratch, the
// work buffers of a B-MSM batch over n_pts points, and what wk holds now
uint64_t msm_table_bytes(uint64_t n_points, uint64_t n_cfg, int fold_c);
uint64_t msm_table_build_bytes(uint64_t n_points);
uint64_t msm_work_bytes(uint64_t n_pts, uint64_t n_cfg, int fold_c, int B, uint64_t v_bytes, int world);
uint64_t msm_work_held(const MsmWork &wk);
// multi-GPU MSMs: the points [p0, p1) rank `rank` of `world` takes
void msm_point_range(uint64_t n, int rank, int world, uint64_t &p0, uint64_t &p1);
// T[k*n + i] = 2^(c*k) P_i, k < W (msm_cfg(n)), affine, in the radix-2^29
// form of field29.cuh (x, y: 14 u32 each, padded to 128 B per point)
void msm_build_table(DevBuf &tab, const uint64_t *d_points, uint64_t n, int c, hipStream_t s);
// n device XYZZ points (24 u64) -> affine (12 u64; infinity -> (0, 0)), synchronous
void xyzz_to_affine_dev(const uint64_t *xyzz, uint64_t n, uint64_t *aff, hipStream_t s);
// the first n (a power of two) commit-key points d_aff (affine, 12 u64 each) in
// the Lagrange basis of the order-n subgroup (lagrange.hip): d_out[i] =
// n_inv sum_j omega_inv^(i j) d_aff[j]; false when the key is degenerate
// (an output at infinity or an exceptional addition); synchronous
bool srs_lagrange(const uint64_t *d_aff, uint64_t n, const Fr &omega_inv, const Fr &n_inv, uint64_t *d_out,
                  hipStream_t s);
// host: XYZZ -> affine Montgomery (inf -> (0, one))
void xyzz_to_affine_host(const uint64_t *xyzz, uint64_t *aff12);
// B points (24 u64 each) -> B affine (12 u64 each), one inversion
void xyzz_to_affine_batch_host(const uint64_t *xyzz, int B, uint64_t *aff12);

// ---- poly / elementwise (poly.hip) ----
void k_from_mont(uint64_t *d, uint64_t n, hipStream_t s);
void k_to_mont(uint64_t *d, uint64_t n, hipStream_t s);
void k_prefix_product(uint64_t *d, uint64_t n, DevBuf &scratch, hipStream_t s);
void k_batch_inverse(uint64_t *d, uint64_t n, DevBuf &scratch, hipStream_t s);
void k_poly_eval(const uint64_t *d, uint64_t n, const Fr &x, DevBuf &scratch, Fr *out,
                 hipStream_t s);
// several polys (same n) at the same point in one launch
void k_poly_eval_multi(const uint64_t *const *polys, int npolys, uint64_t n, const Fr &x,
                       DevBuf &scratch, Fr *out, hipStream_t s);
// several such sets (each its own point), one host round trip for all
struct EvalSet {
    const uint64_t *const *polys;
    int np;
    Fr x;
    Fr *out;
};
void k_poly_eval_sets(const EvalSet *sets, int nsets, uint64_t n, DevBuf &scratch, hipStream_t s);
void k_poly_div_linear(uint64_t *d, uint64_t n, const Fr &z, DevBuf &scratch, hipStream_t s);
// several divisions d_k / (X - z_k) sharing every launch
void k_poly_div_linear_batch(uint64_t *const *d, const Fr *z, int K, uint64_t n, DevBuf &scratch,
                             hipStream_t s);
// d[i] += c z^(len-1-i)
void k_add_powers(uint64_t *d, uint64_t len, const Fr &c, const Fr &z, hipStream_t s);
void k_random_fr(uint64_t *d, uint64_t n, uint64_t seed, hipStream_t s);
// d[i] = c0 * r^i
void k_geometric(uint64_t *d, uint64_t n, const Fr &c0, const Fr &r, hipStream_t s);
void k_srs(uint64_t *d, uint64_t n, const Fr &tau, hipStream_t s);
void k_coset_consts(uint64_t *vh, uint64_t *x, uint32_t lg_n, hipStream_t s);
void k_synth_merkle(int height, const uint64_t *pc_mont_host, const uint64_t *leaves, const uint64_t *blind,
                    uint64_t *nodes, uint64_t *const w[4], uint64_t *const sel[9], uint64_t *const sigma[4],
                    uint64_t n, hipStream_t s);
void k_synth_circuit(uint64_t *const w[4], uint64_t *const sel[9], uint64_t *const sigma[4],
                     uint64_t n, uint64_t n_gates, uint64_t pi_pos, const Fr &pi_mont,
                     hipStream_t s);

}  // namespace pnp
