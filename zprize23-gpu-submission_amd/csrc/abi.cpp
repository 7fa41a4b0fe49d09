// abi.cpp — the extern "C" boundary (include/pnp_plonk.h).
//
// v1 gen_proof keeps the reference's contract (lib/hello.cu:4-6,
// plonk-core/src/lib.rs:237-239): structs by value, ProofC by value,
// synchronous, device 0, print-and-exit on device errors (caffe/common.hpp:
// 23-30).  v2 functions return PNP_* codes and never exit.
#include <algorithm>
#include <dlfcn.h>
#include <array>
#include <atomic>
#include <chrono>
#include <mutex>
#include <set>
#include <thread>
#include <stdarg.h>
#include <stdlib.h>
#include <string.h>
#include "context.h"
#include "ec.cuh"
#include "protocol.h"

namespace pnp {

static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}

// device bytes held by every DevBuf of the process (pnp_hbm_usage)
std::atomic<uint64_t> g_dev_live{0}, g_dev_peak{0};

void DevBuf::alloc(size_t b) {
    release();
    if (b == 0) b = 16;
    // + 64 B past the end: the compiler widens the 8-byte tail load of an F29
    // (ec29.cuh load29: 14 limbs read as 3 x 16 + 8 B) to 16 bytes on the
    // assumption that the element is 16-B aligned; F29s at 56-B strides are only
    // 8-B aligned, so the last one of an array whose end falls on a page boundary
    // would read 8 bytes into the next page (found by tools/ubench_batch_affine
    // faulting on exactly that, DESIGN.md 4 "Fault record")
    hipError_t e = hipMalloc(&p, b + 64);
    if (e != hipSuccess) {
        p = nullptr;
        (void)hipGetLastError();  // clear the sticky out-of-memory status
        set_error("hipMalloc(%zu) failed: %s (%.2f GiB held by this library)", b, hipGetErrorString(e),
                  g_dev_live.load() / 1073741824.0);
        throw Error(PNP_E_NOMEM);
    }
    bytes = b;
    const uint64_t now = g_dev_live.fetch_add(b) + b;
    static const uint64_t trace = [] {  // PNP_HBM_TRACE=bytes: log allocations at least that large
        const char *e = getenv("PNP_HBM_TRACE");
        return e ? strtoull(e, nullptr, 0) : 0ULL;
    }();
    if (trace && b >= trace) {
        Dl_info di{};
        void *ra = __builtin_return_address(0);
        dladdr(ra, &di);
        fprintf(stderr, "pnp hbm: +%zu B (%.3f GiB live) from %s+%#lx\n", b, now / 1073741824.0,
                di.dli_sname ? di.dli_sname : "?", (unsigned long)((char *)ra - (char *)di.dli_saddr));
    }
    uint64_t pk = g_dev_peak.load();
    while (now > pk && !g_dev_peak.compare_exchange_weak(pk, now)) {
    }
}
void DevBuf::release() {
    if (p) {
        (void)hipFree(p);
        g_dev_live.fetch_sub(bytes);
    }
    p = nullptr;
    bytes = 0;
}

// folded table of this rank's point range (msm_point_range) of the first n
// SRS points, rebuilt when n or the sharding changes
const uint64_t *commit_table(pnp_ctx *ctx, uint64_t n) {
    uint64_t p0 = 0, p1 = n;
    if (!ctx->msm.full_table()) msm_point_range(n, ctx->msm.rank, ctx->msm.world, p0, p1);
    if (ctx->ck_table_n != n || ctx->ck_table_p0 != p0 || ctx->ck_table_p1 != p1) {
        ctx->ck_table_n = 0;
        msm_build_table(ctx->ck_table, ctx->ck_dev + 12 * p0, p1 - p0, ctx->msm.fold_c, ctx->stream);
        ctx->ck_table_n = n;
        ctx->ck_table_p0 = p0;
        ctx->ck_table_p1 = p1;
    }
    return ctx->ck_table.u64();
}

// Host -> HBM from the caller's pageable buffers: kStgThreads threads each
// memcpy 8-MiB chunks into two pinned staging buffers of their own and DMA them
// on a stream of their own, so the host copies and the DMAs of several chunks
// overlap (small chunks: pinning the staging memory is a fixed cost of a cold
// call, ~0.4 ms per MiB).  Copies below 4 MiB go through hipMemcpyAsync
// directly.  Measured against HIP's pageable copy (~29-32 GB/s for the 19.5 GB
// prover key of HEIGHT = 15 either way): level on one box, ahead on another
// when the SRS table builds beside the upload (the v1 call one
// proof per process).  PNP_H2D_STAGED=0: hipMemcpyAsync throughout; also the
// fallback when the staging memory cannot be pinned.
static bool h2d_staged_enabled() {
    static const bool on = [] {
        const char *e = getenv("PNP_H2D_STAGED");
        return !(e && atoi(e) == 0);
    }();
    return on;
}
static void h2d_release(pnp_ctx *ctx) {
    for (int k = 0; k < 2 * pnp_ctx::kStgThreads; k++) {
        if (ctx->stg_buf[k]) (void)hipHostFree(ctx->stg_buf[k]);
        if (ctx->stg_ev[k]) (void)hipEventDestroy(ctx->stg_ev[k]);
        ctx->stg_buf[k] = nullptr;
        ctx->stg_ev[k] = nullptr;
    }
    for (int t = 0; t < pnp_ctx::kStgThreads; t++) {
        if (ctx->stg_st[t]) (void)hipStreamDestroy(ctx->stg_st[t]);
        ctx->stg_st[t] = nullptr;
    }
}
void h2d_batch(pnp_ctx *ctx, const std::vector<H2D> &copies) {
    constexpr size_t CH = 8u << 20;
    struct Chunk {
        char *dst;
        const char *src;
        size_t bytes;
    };
    std::vector<Chunk> chunks;
    for (const H2D &c : copies) {
        if (!c.bytes) continue;
        if (!h2d_staged_enabled() || c.bytes < (4u << 20)) {
            PNP_HIP(hipMemcpyAsync(c.dst, c.src, c.bytes, hipMemcpyHostToDevice, ctx->stream));
            continue;
        }
        for (size_t o = 0; o < c.bytes; o += CH)
            chunks.push_back({static_cast<char *>(c.dst) + o, static_cast<const char *>(c.src) + o,
                              std::min(CH, c.bytes - o)});
    }
    PNP_HIP(hipStreamSynchronize(ctx->stream));
    if (chunks.empty()) return;
    constexpr int T = pnp_ctx::kStgThreads;
    if (!ctx->stg_st[T - 1]) {  // the pool, all of it or none (the last member is made last)
        bool ok = true;
        for (int k = 0; k < 2 * T && ok; k++)
            ok = hipHostMalloc(&ctx->stg_buf[k], CH, hipHostMallocDefault) == hipSuccess &&
                 hipEventCreateWithFlags(&ctx->stg_ev[k], hipEventDisableTiming) == hipSuccess;
        for (int t = 0; t < T && ok; t++)
            ok = hipStreamCreateWithFlags(&ctx->stg_st[t], hipStreamNonBlocking) == hipSuccess;
        if (!ok) {
            (void)hipGetLastError();
            h2d_release(ctx);
            for (const Chunk &c : chunks)
                PNP_HIP(hipMemcpyAsync(c.dst, c.src, c.bytes, hipMemcpyHostToDevice, ctx->stream));
            PNP_HIP(hipStreamSynchronize(ctx->stream));
            return;
        }
    }
    std::atomic<size_t> next{0};
    std::atomic<int> failed{0};
    auto worker = [&](int t) {
        try {
            PNP_HIP(hipSetDevice(ctx->device));
            int use = 0;
            for (size_t j; (j = next.fetch_add(1)) < chunks.size() && !failed.load();) {
                const int k = 2 * t + use;
                use ^= 1;
                PNP_HIP(hipEventSynchronize(ctx->stg_ev[k]));  // this buffer's previous DMA has landed
                memcpy(ctx->stg_buf[k], chunks[j].src, chunks[j].bytes);
                PNP_HIP(hipMemcpyAsync(chunks[j].dst, ctx->stg_buf[k], chunks[j].bytes, hipMemcpyHostToDevice,
                                       ctx->stg_st[t]));
                PNP_HIP(hipEventRecord(ctx->stg_ev[k], ctx->stg_st[t]));
            }
            PNP_HIP(hipStreamSynchronize(ctx->stg_st[t]));
        } catch (...) {
            failed.store(1);
            (void)hipStreamSynchronize(ctx->stg_st[t]);  // no DMA of this thread outlives the call
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < T; t++) th.emplace_back(worker, t);
    worker(0);
    for (auto &x : th) x.join();
    if (failed.load()) {
        set_error("host -> HBM staged upload failed");
        throw Error(PNP_E_DEVICE);
    }
}

void ck_derived_reset(pnp_ctx *ctx) {
    ctx->ck_table_n = 0;
    ctx->ck_table.release();
    ctx->lag_n = 0;
    ctx->lag_ok = false;
    ctx->lag_points.release();
    ctx->lag_table_n = 0;
    ctx->lag_table.release();
    wire_bases_reset(ctx);
}

// every rank's verdict on a step that may fail on some rank only (an optional
// table that did not fit its HBM): true when it succeeded on all of them
bool all_ranks_ok(pnp_ctx *ctx, bool mine) {
    if (ctx->msm.world <= 1 || !ctx->msm.allgather) return mine;
    const uint64_t w = mine ? 1 : 0;
    for (uint64_t v : rank_allgather(ctx->msm, ctx->stream, &w, 1, PNP_EX_TAG_STATUS))
        if (!v) return false;
    return true;
}

// ---- background table build (context.h pnp_ctx::bg) ----
thread_local bool t_bg_build = false;
static thread_local std::atomic<bool> *t_bg_cancel = nullptr;

void bg_step(hipStream_t s) {
    if (!t_bg_build) return;
    PNP_HIP(hipStreamSynchronize(s));
    if (t_bg_cancel && t_bg_cancel->load()) {
        set_error("background table build cancelled");
        throw Error(PNP_E_DEVICE);
    }
}

hipStream_t tables_stream(pnp_ctx *ctx) { return t_bg_build ? ctx->bg_stream : ctx->stream; }

// contexts whose builder may still run at process exit (the v1 symbol's
// context is never destroyed): stopped and joined before the HIP runtime's
// own exit handlers run (registered after them, so called first)
static std::mutex g_bg_mu;
static std::set<pnp_ctx *> g_bg_live;
static void bg_atexit() {
    std::vector<pnp_ctx *> live;
    {
        std::lock_guard<std::mutex> lk(g_bg_mu);
        live.assign(g_bg_live.begin(), g_bg_live.end());
    }
    for (pnp_ctx *c : live) tables_cancel(c);
}

static void bg_build(pnp_ctx *ctx, uint64_t n) {
    t_bg_build = true;
    t_bg_cancel = &ctx->bg_cancel;
    bool groups_started = false;
    try {
        PNP_HIP(hipSetDevice(ctx->device));
        if (lagrange_table(ctx, n)) {
            groups_started = true;
            wire_bases_build(ctx, n);
        }
        PNP_HIP(hipStreamSynchronize(ctx->bg_stream));
    } catch (...) {
        // cancelled (a key load or the context's end) or failed: a half-built
        // group set is dropped (the next deferring proof starts a new build,
        // which resumes from the finished Lagrange parts); a failure leaves
        // the proofs without what is not complete
        (void)hipStreamSynchronize(ctx->bg_stream);
        if (groups_started) wire_bases_reset(ctx);
        if (!ctx->bg_cancel.load()) {
            ctx->hbm_lag_off = !(ctx->lag_ok && ctx->lag_table_n == n);
            ctx->hbm_groups_off = true;
        }
    }
    ctx->bg_state.store(2, std::memory_order_release);
}

bool tables_bg_enabled() {
    static const bool on = [] {
        const char *e = getenv("PNP_DEFER_BG");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

void tables_start_background(pnp_ctx *ctx, uint64_t n) {
    if (ctx->msm.world > 1 || ctx->bg.joinable() || !tables_bg_enabled()) return;
    if (!ctx->bg_stream) {
        int lo = 0, hi = 0;
        PNP_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
        PNP_HIP(hipStreamCreateWithPriority(&ctx->bg_stream, hipStreamNonBlocking, lo));
    }
    // the builder reads what this proof's stream wrote (the key uploads)
    PNP_HIP(hipStreamSynchronize(ctx->stream));
    {
        static std::once_flag once;
        std::call_once(once, [] { atexit(bg_atexit); });
        std::lock_guard<std::mutex> lk(g_bg_mu);
        g_bg_live.insert(ctx);
    }
    ctx->bg_cancel.store(false);
    ctx->bg_state.store(1, std::memory_order_release);
    ctx->bg = std::thread(bg_build, ctx, n);
}

static void bg_join(pnp_ctx *ctx) {
    if (ctx->bg.joinable()) ctx->bg.join();
    ctx->bg_state.store(0);
    std::lock_guard<std::mutex> lk(g_bg_mu);
    g_bg_live.erase(ctx);
}

bool tables_busy(pnp_ctx *ctx) {
    if (t_bg_build) return false;
    const int st = ctx->bg_state.load(std::memory_order_acquire);
    if (st == 2) bg_join(ctx);
    return st == 1;
}

void tables_wait(pnp_ctx *ctx) {
    if (!t_bg_build && ctx->bg.joinable()) bg_join(ctx);
}

void tables_cancel(pnp_ctx *ctx) {
    if (t_bg_build || !ctx->bg.joinable()) return;
    ctx->bg_cancel.store(true);
    bg_join(ctx);
    ctx->bg_cancel.store(false);
}

bool lagrange_enabled() {
    static const bool enabled = [] {
        const char *e = getenv("PNP_LAGRANGE");
        return !e || atoi(e) != 0;
    }();
    return enabled;
}

const uint64_t *lagrange_table(pnp_ctx *ctx, uint64_t n) {
    if (!lagrange_enabled() || ctx->hbm_lag_off || n < 2 || (n & (n - 1)) || n > ctx->ck_points) return nullptr;
    if (tables_busy(ctx)) return nullptr;  // being built in the background: commit without it
    uint64_t p0 = 0, p1 = n;
    if (!ctx->msm.full_table()) msm_point_range(n, ctx->msm.rank, ctx->msm.world, p0, p1);
    // a deferring proof uses the table only if it is there
    if (ctx->defer_now && !t_bg_build &&
        !(ctx->lag_n == n && ctx->lag_ok && ctx->lag_table_n == n && ctx->lag_table_p0 == p0 &&
          ctx->lag_table_p1 == p1)) {
        if (!(ctx->lag_n == n && !ctx->lag_ok)) ctx->tables_wanted = true;  // (not a degenerate key)
        return nullptr;
    }
    // (re)built on the same call on every rank (same key and call sequence):
    // a rank whose HBM could not hold it makes every rank go without
    bool built = false, fits = true;
    try {
        if (ctx->lag_n != n) {
            built = true;
            ctx->lag_table_n = 0;
            ctx->lag_table.release();
            ctx->lag_n = 0;
            ctx->lag_points.alloc(n * 96);
            uint32_t lg = 0;
            while ((1ULL << lg) < n) lg++;
            ctx->lag_ok = srs_lagrange(ctx->ck_dev, n, inverse(root_of_unity(lg)), inverse(fr_from_u64(n)),
                                       ctx->lag_points.u64(), tables_stream(ctx));
            ctx->lag_n = n;
            if (!ctx->lag_ok) ctx->lag_points.release();
        }
        if (ctx->lag_ok && (ctx->lag_table_n != n || ctx->lag_table_p0 != p0 || ctx->lag_table_p1 != p1)) {
            built = true;
            ctx->lag_table_n = 0;
            msm_build_table(ctx->lag_table, ctx->lag_points.u64() + 12 * p0, p1 - p0, ctx->msm.fold_c,
                            tables_stream(ctx));
            ctx->lag_table_n = n;
            ctx->lag_table_p0 = p0;
            ctx->lag_table_p1 = p1;
        }
    } catch (const Error &e) {
        if (e.code != PNP_E_NOMEM) throw;
        fits = false;
    }
    if (built && !all_ranks_ok(ctx, fits)) fits = false;
    if (!fits) {  // commit from coefficients (prover.cpp), on every rank
        ctx->lag_points.release();
        ctx->lag_table.release();
        ctx->lag_table_n = 0;
        ctx->lag_n = n;
        ctx->lag_ok = false;
        ctx->hbm_lag_off = true;
        return nullptr;
    }
    if (!ctx->lag_ok) return nullptr;
    return ctx->lag_table.u64();
}

// ---- HBM budget (key load) ----
// Upper bounds of what a proof at domain n allocates on this rank, by part:
// the mandatory working set (per-proof buffers, NTT tables, the commit key's
// folded table and its build, the MSM work of the largest batch) and the two
// optional derived tables (the Lagrange basis with its table; the
// copy-constraint groups with theirs), each minus what is already held.
// Checked against the measured peak by tests/test_gpu_hbm.py.
static uint64_t map_bytes(const std::map<std::string, DevBuf> &m) {
    uint64_t b = 0;
    for (const auto &kv : m) b += kv.second.bytes;
    return b;
}
static uint64_t map_bytes(const std::map<uint32_t, DevBuf> &m) {
    uint64_t b = 0;
    for (const auto &kv : m) b += kv.second.bytes;
    return b;
}
HbmPlan hbm_plan(pnp_ctx *ctx, uint64_t n) {
    HbmPlan p;
    const MsmWork &wk = ctx->msm;
    const int world = wk.world;
    const bool full = wk.full_table();
    const uint64_t per = (n + world - 1) / world;  // this rank's point range (at most)
    const uint64_t n_tab = full ? n : per;
    const bool dist = ctx->pk_nb < 8;
    const uint64_t len = dist ? per : n, NB = (uint64_t)ctx->pk_nb * n, N8 = 8 * n;
    const bool lookups = !ctx->pk_qlookup_zero;
    // per-proof buffers (prover.cpp ctx->buf): 21 of n always (wires, their
    // coefficients, the lookup / grand-product vectors), the PI and L1
    // polynomials when not in closed form; 11 of the coefficient range (t
    // chunks, linearisation, opening combinations); of the rank's blocks: the
    // wire / z / z2 LDEs and t (7), the PI term's 1 / (x - w^pos), the lookup
    // LDEs, the L1 / PI LDEs when not in closed form; the batch-inverse /
    // scan scratch (about one vector of the longest length)
    const bool closed = ctx->pk_std_coset;
    const uint64_t work = 32 * (21 * n + (closed ? 0 : 2 * n) + 11 * len +
                                NB * (8 + (lookups ? 4 : 0) + (closed ? 0 : 2)) + std::max(n, NB) * 9 / 8);
    const uint64_t work_held = map_bytes(ctx->work) + ctx->scratch_a.bytes + ctx->scratch_b.bytes + ctx->pk_pinv.bytes;
    // NTT tables: twiddles of n (both directions), the block twists (forward,
    // inverse, x32) of the 8n coset; with PNP_NTT29 their 2^261 forms
    static const bool ntt29 = [] {
        const char *e = getenv("PNP_NTT29");
        return e && atoi(e) != 0;
    }();
    // (+ the dense twiddle rows of both directions, 2 x (n - 1) entries)
    const uint64_t ntt = 32 * n + 64 * n + 3 * 32 * N8 + (ntt29 ? 36 * n / 2 * 2 + 3 * 36 * N8 : 0);
    // (the 8n LDE twist of pnp_coset_lde8 is not a proof's: not counted as held)
    const uint64_t ntt_held = map_bytes(ctx->ntt.fwd) + map_bytes(ctx->ntt.inv) + map_bytes(ctx->ntt.fwd_rows) +
                              map_bytes(ctx->ntt.inv_rows) + map_bytes(ctx->ntt.blk_twist) +
                              map_bytes(ctx->ntt.blk_twist_inv) + map_bytes(ctx->ntt.fwd29) +
                              map_bytes(ctx->ntt.inv29) + map_bytes(ctx->ntt.blk_twist29) +
                              map_bytes(ctx->ntt.blk_twist_inv29) + map_bytes(ctx->ntt.blk_twist32) +
                              map_bytes(ctx->ntt.blk_twist32_29);
    const uint64_t ck_tab = msm_table_bytes(n_tab, n, wk.fold_c);
    const uint64_t msm = msm_work_bytes(per, n, wk.fold_c, 9, wk.v_bytes, world);
    const uint64_t held = work_held + ntt_held + ctx->ck_table.bytes + msm_work_held(wk);
    const uint64_t total = work + ntt + ck_tab + msm;
    p.mandatory = total > held ? total - held : 0;
    p.t_mand = ctx->ck_table.bytes ? 0 : msm_table_build_bytes(n_tab);
    // the Lagrange basis (n affine points) + its folded table; its build:
    // the radix-2^29 layer array, the window tables, the XYZZ output
    const uint64_t lag = n * 96 + msm_table_bytes(n_tab, n, wk.fold_c);
    const uint64_t lag_held = ctx->lag_points.bytes + ctx->lag_table.bytes;
    const bool lag_built = ctx->lag_n == n && (!ctx->lag_ok || ctx->lag_table_n == n);
    p.lag = lag_built ? 0 : lag > lag_held ? lag - lag_held : 0;
    if (p.lag) p.t_lag = n * (224 + 16 + 192 + 48) + std::min<uint64_t>(n / 2, 1ULL << 18) * 15 * 224;
    // the copy-constraint groups: 5 segments of n slots (this rank's slice in
    // point-range mode), their folded table, the group maps and scalars, the
    // sigma copy; the build: sort keys and labels, XYZZ bases, affine points
    const uint64_t seg = full ? n : (world > 1 ? per : n);
    const uint64_t grp = msm_table_bytes(5 * seg, n, wk.fold_c) + 5 * n * (4 + 4 + 32) + 4 * n * 32;
    uint64_t grp_held = ctx->wb.table.bytes + ctx->wb.sigma.bytes + ctx->wb.flag.bytes;
    for (int j = 0; j < 5; j++) grp_held += ctx->wb.grp[j].bytes + ctx->wb.rep[j].bytes + ctx->wb.scal[j].bytes;
    const bool grp_built = ctx->wb.built && ctx->wb.n == n;
    p.groups = grp_built ? 0 : grp > grp_held ? grp - grp_held : 0;
    if (p.groups)
        p.t_groups = 4 * n * (32 + 8 + 8 + 4 + 4 + 4 + 4 + 4 + 4) + 5 * n * 192 + 5 * seg * (192 + 96) +
                     msm_table_build_bytes(5 * seg);
    p.transient = std::max({p.t_mand, p.t_lag, p.t_groups});
    return p;
}

// The HBM budget, checked by the first proof after a key load (by then the
// caller has released what it no longer needs, e.g. its own 8n key arrays
// once the context holds their block copies): the rank's share of its GPU's
// free HBM (ranks on one device split it) against hbm_plan.  The optional
// tables that do not fit are switched off on every rank (the proof bytes do
// not change); when even the mandatory part does not fit, every rank's proof
// fails with PNP_E_NOMEM before any work, with a message naming the rank and
// the bytes, instead of one rank running out of memory mid-proof and its
// peers failing in an exchange.  PNP_HBM_LIMIT (bytes) caps the budget (tests).
static uint64_t device_key(int dev) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof bus, dev) != hipSuccess) snprintf(bus, sizeof bus, "dev%d", dev);
    uint64_t h = 1469598103934665603ULL;  // FNV-1a
    for (const char *c = bus; *c; c++) h = (h ^ (uint8_t)*c) * 1099511628211ULL;
    return h;
}
void hbm_budget(pnp_ctx *ctx) {
    MsmWork &wk = ctx->msm;
    const int W = wk.world > 1 && wk.allgather ? wk.world : 1;
    uint64_t share = 1;
    if (W > 1) {  // (also the barrier after which every rank's key load has allocated)
        const uint64_t id = device_key(ctx->device);
        share = 0;
        for (uint64_t v : rank_allgather(wk, ctx->stream, &id, 1, PNP_EX_TAG_DEVICE)) share += v == id;
    }
    size_t fr = 0, tot = 0;
    PNP_HIP(hipMemGetInfo(&fr, &tot));
    uint64_t budget = fr / std::max<uint64_t>(share, 1);
    if (const char *e = getenv("PNP_HBM_LIMIT")) {
        const uint64_t lim = strtoull(e, nullptr, 0), live = g_dev_live.load();
        budget = std::min<uint64_t>(budget, lim > live ? lim - live : 0);
    }
    const HbmPlan p = hbm_plan(ctx, ctx->pk_n);
    // each optional table with the largest build scratch among what is built
    const uint64_t base = p.mandatory + p.t_mand;
    const uint64_t with_lag = p.mandatory + p.lag + std::max(p.t_mand, p.t_lag);
    const uint64_t with_groups = with_lag - std::max(p.t_mand, p.t_lag) + p.groups +
                                 std::max({p.t_mand, p.t_lag, p.t_groups});
    // PNP_HBM_BUDGET=0: the mandatory part is an upper bound (up to ~3x the
    // measured peak, test_gpu_hbm.py), so a caller that knows better lets the
    // real allocations decide; the optional tables are still sized here
    static const bool hard = [] {
        const char *e = getenv("PNP_HBM_BUDGET");
        return !(e && atoi(e) == 0);
    }();
    constexpr int K = 6;
    uint64_t mine[K];
    mine[0] = !hard || base <= budget;
    mine[1] = lagrange_enabled() && with_lag <= budget;
    mine[2] = mine[1] && wire_groups_enabled() && with_groups <= budget;
    mine[3] = base;
    mine[4] = budget;
    // PNP_DEFER_TABLES is read per process: the ranks defer together or not
    // at all (a deferring rank would skip the table builds' status exchange)
    mine[5] = ctx->defer_tables;
    std::vector<uint64_t> all(mine, mine + K);
    if (W > 1) all = rank_allgather(wk, ctx->stream, mine, K, PNP_EX_TAG_STATUS);
    bool ok = true, lag = true, groups = true, defer = true;
    int bad = -1;
    for (int r = 0; r < W; r++) {
        if (!all[K * r] && bad < 0) bad = r;
        ok &= all[K * r] != 0;
        lag &= all[K * r + 1] != 0;
        groups &= all[K * r + 2] != 0;
        defer &= all[K * r + 5] != 0;
    }
    ctx->hbm_lag_off = !lag;
    ctx->hbm_groups_off = !groups;
    if (!defer) {
        ctx->defer_tables = false;
        ctx->defer_now = false;
    }
    if (!ok) {
        set_error("HBM budget: rank %d of %d needs %.2f GiB more for a proof at n = %llu, %.2f GiB free to it "
                  "(%llu rank(s) on this rank's GPU; PNP_HBM_BUDGET=0 lets the allocations decide)", bad, W,
                  all[K * bad + 3] / 1073741824.0, (unsigned long long)ctx->pk_n, all[K * bad + 4] / 1073741824.0,
                  (unsigned long long)share);
        throw Error(PNP_E_NOMEM);
    }
}

void commit_evals_batch(pnp_ctx *ctx, const uint64_t *const *d_evals, int B, uint64_t n, CommitmentC *const *out) {
    const uint64_t *table = lagrange_table(ctx, n);
    if (!table) {
        set_error("commit from evaluations: no Lagrange-basis key of size %llu", (unsigned long long)n);
        throw Error(PNP_E_ARG);
    }
    std::vector<uint64_t> xyzz((size_t)B * 24);
    msm_run_batch(ctx->msm, ctx->lag_points.u64(), d_evals, B, n, xyzz.data(), ctx->stream, table, false);
    std::vector<uint64_t> aff((size_t)B * 12);
    xyzz_to_affine_batch_host(xyzz.data(), B, aff.data());
    for (int b = 0; b < B; b++) {
        memcpy(out[b]->x, &aff[12 * b], 48);
        memcpy(out[b]->y, &aff[12 * b + 6], 48);
    }
}

void commit_affine(pnp_ctx *ctx, const uint64_t *d_scalars, uint64_t n, CommitmentC *out) {
    uint64_t xyzz[24], aff[12];
    msm_run(ctx->msm, ctx->ck_dev, d_scalars, n, xyzz, ctx->stream, commit_table(ctx, n));
    xyzz_to_affine_host(xyzz, aff);
    memcpy(out->x, aff, 48);
    memcpy(out->y, aff + 6, 48);
}

hipEvent_t KernelTimer::get() {
    if (!pool.empty()) {
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
    }
    hipEvent_t e;
    PNP_HIP(hipEventCreate(&e));
    return e;
}
void KernelTimer::begin(const char *, hipStream_t s, hipEvent_t &e0) {
    if (!enabled) return;
    e0 = get();
    PNP_HIP(hipEventRecord(e0, s));
}
void KernelTimer::end(const char *name, hipStream_t s, hipEvent_t e0, double bytes) {
    if (!enabled || !e0) return;
    hipEvent_t e1 = get();
    PNP_HIP(hipEventRecord(e1, s));
    pending.push_back({name, e0, e1, bytes});
}
void KernelTimer::collect() {
    for (auto &p : pending) {
        float ms = 0;
        PNP_HIP(hipEventSynchronize(p.e1));  // (no-op once the stream has drained)
        PNP_HIP(hipEventElapsedTime(&ms, p.e0, p.e1));
        auto &st = stats[p.name];
        st.ms += ms;
        st.bytes += p.bytes;
        st.launches += 1;
        pool.push_back(p.e0);
        pool.push_back(p.e1);
    }
    pending.clear();
}

void commit_affine_batch(pnp_ctx *ctx, const uint64_t *const *d_scalars, int B, uint64_t n,
                         CommitmentC *const *out, bool local) {
    std::vector<uint64_t> xyzz((size_t)B * 24);
    msm_run_batch(ctx->msm, ctx->ck_dev, d_scalars, B, n, xyzz.data(), ctx->stream,
                  commit_table(ctx, n), local);
    std::vector<uint64_t> aff((size_t)B * 12);
    xyzz_to_affine_batch_host(xyzz.data(), B, aff.data());
    for (int b = 0; b < B; b++) {
        memcpy(out[b]->x, &aff[12 * b], 48);
        memcpy(out[b]->y, &aff[12 * b + 6], 48);
    }
}

}  // namespace pnp

hipStream_t pnp_ctx::side_stream() {
    if (!stream_lo) {
        int lo = 0, hi = 0;
        PNP_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));  // lo = least priority
        // PNP_SIDE_PRIORITY=hi: the side stream's transforms ahead of the main
        // stream's MSM (experiments)
        const char *pe = getenv("PNP_SIDE_PRIORITY");
        const bool side_hi = pe && !strcmp(pe, "hi");
        PNP_HIP(hipStreamCreateWithPriority(&stream_lo, hipStreamNonBlocking, side_hi ? hi : lo));
        for (hipEvent_t *e : {&ev_fork, &ev_w8, &ev_z8})
            PNP_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
    }
    return stream_lo;
}

uint64_t *pnp_ctx::buf(const std::string &name, size_t elems_fr) {
    auto &b = work[name];
    if (b.bytes < elems_fr * 32) b.alloc(elems_fr * 32);
    return b.u64();
}

using namespace pnp;

#define PNP_TRY(...)                                   \
    try {                                              \
        __VA_ARGS__;                                   \
        return PNP_OK;                                 \
    } catch (const Error &e) {                         \
        return e.code;                                 \
    } catch (const std::exception &e) {                \
        set_error("exception: %s", e.what());          \
        return PNP_E_DEVICE;                           \
    }

extern "C" {

const char *pnp_last_error(void) { return g_err; }

int pnp_ctx_create(int device, pnp_ctx **out) {
    if (!out) return PNP_E_ARG;
    pnp_ctx *c = new pnp_ctx();
    try {
        c->device = device;
        if (const char *e = getenv("PNP_FOLD_C")) c->msm.fold_c = atoi(e);  // experiments
        if (const char *e = getenv("PNP_DEFER_TABLES")) c->defer_tables = atoi(e) != 0 ? 1 : 0;
        PNP_HIP(hipSetDevice(device));
        PNP_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    } catch (const Error &e) {
        delete c;
        return e.code;
    }
    *out = c;
    return PNP_OK;
}

void pnp_ctx_destroy(pnp_ctx *ctx) {
    if (!ctx) return;
    tables_cancel(ctx);
    if (ctx->bg_stream) (void)hipStreamDestroy(ctx->bg_stream);
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->msm.s2) {
        (void)hipStreamSynchronize(ctx->msm.s2);
        (void)hipStreamDestroy(ctx->msm.s2);
    }
    for (hipEvent_t e : ctx->msm.ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->stream_lo) {
        (void)hipStreamSynchronize(ctx->stream_lo);
        (void)hipStreamDestroy(ctx->stream_lo);
        for (hipEvent_t e : {ctx->ev_fork, ctx->ev_w8, ctx->ev_z8}) (void)hipEventDestroy(e);
    }
    (void)hipStreamDestroy(ctx->stream);
    h2d_release(ctx);
    for (hipEvent_t e : ctx->ktimer.pool) (void)hipEventDestroy(e);
    for (auto &p : ctx->ktimer.pending) {
        (void)hipEventDestroy(p.e0);
        (void)hipEventDestroy(p.e1);
    }
    delete ctx;
}

int pnp_kernel_timing(pnp_ctx *ctx, int enable) {
    if (!ctx) return PNP_E_ARG;
    ctx->ktimer.enabled = enable != 0;
    ctx->msm.timer = enable ? &ctx->ktimer : nullptr;
    if (enable) ctx->ktimer.stats.clear();
    return PNP_OK;
}

int pnp_kernel_stats(pnp_ctx *ctx, const char *name, double *total_ms, int *launches) {
    if (!ctx || !name) return PNP_E_ARG;
    try {
        ctx->ktimer.collect();  // operator calls leave their events pending
    } catch (const Error &e) {
        return e.code;
    }
    auto it = ctx->ktimer.stats.find(name);
    if (total_ms) *total_ms = it == ctx->ktimer.stats.end() ? 0.0 : it->second.ms;
    if (launches) *launches = it == ctx->ktimer.stats.end() ? 0 : it->second.launches;
    return PNP_OK;
}

int pnp_kernel_bytes(pnp_ctx *ctx, const char *name, double *bytes) {
    if (!ctx || !name || !bytes) return PNP_E_ARG;
    auto it = ctx->ktimer.stats.find(name);
    *bytes = it == ctx->ktimer.stats.end() ? 0.0 : it->second.bytes;
    return PNP_OK;
}

int pnp_set_msm_shard(pnp_ctx *ctx, int rank, int world, pnp_allgather_fn allgather, void *user,
                      uint64_t *d_xbuf, uint64_t xbuf_bytes) {
    if (!ctx || world < 1 || rank < 0 || rank >= world) return PNP_E_ARG;
    if (world > 1 && (!allgather || !d_xbuf)) return PNP_E_ARG;
    // a background table build reads msm.world / rank / allgather (all_ranks_ok)
    // and writes the tables whose point ranges these settings decide: stop it
    // first (the next deferring proof starts a new one)
    tables_cancel(ctx);
    ctx->msm.rank = world > 1 ? rank : 0;
    ctx->msm.world = world;
    ctx->msm.allgather = world > 1 ? allgather : nullptr;
    ctx->msm.user = user;
    ctx->msm.xbuf = world > 1 ? d_xbuf : nullptr;
    ctx->msm.xbuf_bytes = world > 1 ? xbuf_bytes : 0;
    return PNP_OK;
}

int pnp_set_exchange_a2a(pnp_ctx *ctx, pnp_alltoall_fn alltoall, void *user, uint64_t *d_a2a,
                         uint64_t a2a_bytes) {
    if (!ctx || (alltoall && !d_a2a)) return PNP_E_ARG;
    tables_cancel(ctx);  // (as pnp_set_msm_shard)
    ctx->msm.alltoall = alltoall;
    ctx->msm.a2a_user = user;
    ctx->msm.a2a = alltoall ? d_a2a : nullptr;
    ctx->msm.a2a_bytes = alltoall ? a2a_bytes : 0;
    return PNP_OK;
}

int pnp_set_exchange_v(pnp_ctx *ctx, pnp_alltoallv_fn alltoallv, void *user, uint64_t *d_send,
                       uint64_t *d_recv, uint64_t capacity_bytes) {
    if (!ctx || (alltoallv && (!d_send || !d_recv || capacity_bytes < 8))) return PNP_E_ARG;
    tables_cancel(ctx);  // the builder may be writing lag_table, released below
    ctx->msm.alltoallv = alltoallv;
    ctx->msm.v_user = user;
    ctx->msm.v_send = alltoallv ? d_send : nullptr;
    ctx->msm.v_recv = alltoallv ? d_recv : nullptr;
    ctx->msm.v_bytes = alltoallv ? capacity_bytes : 0;
    // the folded tables' point ranges change (the Lagrange points stay)
    ctx->ck_table_n = 0;
    ctx->ck_table.release();
    ctx->lag_table_n = 0;
    ctx->lag_table.release();
    return PNP_OK;
}

int pnp_set_exchange_ordered(pnp_ctx *ctx, int ordered) {
    if (!ctx) return PNP_E_ARG;
    ctx->msm.ordered = ordered != 0;
    return PNP_OK;
}

int pnp_ctx_stream(pnp_ctx *ctx, void **stream) {
    if (!ctx || !stream) return PNP_E_ARG;
    *stream = ctx->stream;
    return PNP_OK;
}

int pnp_sync(pnp_ctx *ctx) {
    if (!ctx) return PNP_E_ARG;
    // (and the background table build: pnp_sync waits for all of the context's work)
    PNP_TRY({
        tables_wait(ctx);
        PNP_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int pnp_ntt(pnp_ctx *ctx, uint64_t *d, uint32_t lg_n, int inverse, int coset) {
    if (!ctx || !d || lg_n > 28) return PNP_E_ARG;
    // timed (pnp_kernel_timing): "ntt", credited 2 x 32 B per element (one
    // read, one write: SURVEY 8(d)'s algorithmic bytes of a transform)
    PNP_TRY({
        hipEvent_t e0 = nullptr;
        ctx->ktimer.begin("ntt", ctx->stream, e0);
        ntt_run(ctx->ntt, d, lg_n, inverse != 0, coset != 0, ctx->stream);
        ctx->ktimer.end("ntt", ctx->stream, e0, 64.0 * (double)(1ULL << lg_n));
    });
}

int pnp_coset_lde8(pnp_ctx *ctx, const uint64_t *in, uint64_t *out8, uint32_t lg_n) {
    if (!ctx || !in || !out8 || lg_n > 25) return PNP_E_ARG;
    PNP_TRY(coset_lde8(ctx->ntt, in, out8, lg_n, ctx->stream));
}

int pnp_commit(pnp_ctx *ctx, const uint64_t *d_points, const uint64_t *d_scalars, uint64_t n,
               CommitmentC *out) {
    if (!ctx || !out || (n && (!d_points || !d_scalars))) return PNP_E_ARG;
    PNP_TRY({
        uint64_t xyzz[24], aff[12];
        msm_run(ctx->msm, d_points, d_scalars, n, xyzz, ctx->stream);
        xyzz_to_affine_host(xyzz, aff);
        memcpy(out->x, aff, 48);
        memcpy(out->y, aff + 6, 48);
    });
}

int pnp_commit_ck(pnp_ctx *ctx, const uint64_t *d_scalars, uint64_t n, CommitmentC *out) {
    if (!ctx || !out || (n && !d_scalars)) return PNP_E_ARG;
    if (!ctx->ck_loaded) {
        set_error("commit key not loaded");
        return PNP_E_NOKEY;
    }
    if (n > ctx->ck_points) {
        set_error("commit key has %llu points, need %llu", (unsigned long long)ctx->ck_points,
                  (unsigned long long)n);
        return PNP_E_ARG;
    }
    // timed (pnp_kernel_timing): "msm", the whole MSM (digits, sort,
    // accumulation, bucket reduction, result), credited n (96 + 32) B (every
    // point and scalar once); the folded table is built first
    PNP_TRY({
        commit_table(ctx, n);
        hipEvent_t e0 = nullptr;
        ctx->ktimer.begin("msm", ctx->stream, e0);
        commit_affine(ctx, d_scalars, n, out);
        ctx->ktimer.end("msm", ctx->stream, e0, 128.0 * (double)n);
    });
}

int pnp_commit_evals(pnp_ctx *ctx, const uint64_t *d_evals, uint64_t n, CommitmentC *out) {
    if (!ctx || !out || !d_evals) return PNP_E_ARG;
    tables_wait(ctx);  // (a background build of the Lagrange basis finishes first)
    if (!ctx->ck_loaded) {
        set_error("commit key not loaded");
        return PNP_E_NOKEY;
    }
    if (n < 2 || (n & (n - 1)) || n > ctx->ck_points) {
        set_error("commit from evaluations: n = %llu must be a power of two <= %llu", (unsigned long long)n,
                  (unsigned long long)ctx->ck_points);
        return PNP_E_ARG;
    }
    PNP_TRY({
        CommitmentC *o[1] = {out};
        const uint64_t *e[1] = {d_evals};
        commit_evals_batch(ctx, e, 1, n, o);
    });
}

int pnp_hbm_usage(pnp_ctx *ctx, uint64_t out[6]) {
    if (!out) return PNP_E_ARG;
    PNP_TRY({
        if (ctx) tables_wait(ctx);
        out[0] = g_dev_live.load();
        out[1] = g_dev_peak.exchange(out[0]);  // the peak since the previous call
        pnp::HbmPlan p;
        if (ctx && ctx->pk_loaded) p = pnp::hbm_plan(ctx, ctx->pk_n);
        out[2] = p.mandatory;
        out[3] = p.lag;
        out[4] = p.groups;
        out[5] = p.transient;
    });
}

int pnp_commit_segments(pnp_ctx *ctx, const uint64_t *d_points, uint64_t n_points, int B, const uint64_t *seg_off,
                        const uint64_t *const *d_scalars, uint64_t n, CommitmentC *out) {
    if (!ctx || !out || !seg_off || !d_scalars || B < 1 || B > 16 || (n_points && !d_points)) return PNP_E_ARG;
    for (int b = 0; b < B; b++) {
        if ((n && !d_scalars[b]) || seg_off[b] > n_points || n > n_points - seg_off[b]) {
            set_error("commit segments: MSM %d covers points [%llu, %llu) of %llu", b,
                      (unsigned long long)seg_off[b], (unsigned long long)(seg_off[b] + n),
                      (unsigned long long)n_points);
            return PNP_E_ARG;
        }
    }
    if (ctx->msm.world > 1) {
        set_error("commit segments: single-GPU operator");
        return PNP_E_ARG;
    }
    PNP_TRY({
        std::vector<uint64_t> xyzz((size_t)B * 24), aff((size_t)B * 12);
        if (n != 0) {  // n = 0: every sum is infinity (ZZ = 0)
            DevBuf tab;
            msm_build_table(tab, d_points, n_points, msm_fold_c(n, ctx->msm.fold_c), ctx->stream);
            MsmSegs segs;
            segs.n_table = n_points;
            for (int b = 0; b < B; b++) segs.off[b] = seg_off[b];
            segs.c = msm_fold_c(n, ctx->msm.fold_c);
            msm_run_batch(ctx->msm, nullptr, d_scalars, B, n, xyzz.data(), ctx->stream, tab.u64(), false, &segs);
        }
        xyzz_to_affine_batch_host(xyzz.data(), B, aff.data());
        for (int b = 0; b < B; b++) {
            memcpy(out[b].x, &aff[12 * b], 48);
            memcpy(out[b].y, &aff[12 * b + 6], 48);
        }
    });
}

int pnp_poly_eval(pnp_ctx *ctx, const uint64_t *d, uint64_t n, const uint64_t x[4], uint64_t out[4]) {
    if (!ctx || !d || !x || !out) return PNP_E_ARG;
    PNP_TRY({
        Fr r;
        k_poly_eval(d, n, from_u64_limbs<FrP>(x), ctx->scratch_a, &r, ctx->stream);
        to_u64_limbs(r, out);
    });
}

int pnp_poly_div_linear(pnp_ctx *ctx, uint64_t *d, uint64_t n, const uint64_t z[4]) {
    if (!ctx || !d || !z) return PNP_E_ARG;
    PNP_TRY(k_poly_div_linear(d, n, from_u64_limbs<FrP>(z), ctx->scratch_a, ctx->stream));
}

int pnp_prefix_product(pnp_ctx *ctx, uint64_t *d, uint64_t n) {
    if (!ctx || !d) return PNP_E_ARG;
    PNP_TRY(k_prefix_product(d, n, ctx->scratch_a, ctx->stream));
}

int pnp_batch_inverse(pnp_ctx *ctx, uint64_t *d, uint64_t n) {
    if (!ctx || !d) return PNP_E_ARG;
    PNP_TRY(k_batch_inverse(d, n, ctx->scratch_a, ctx->stream));
}

int pnp_synth_random_fr(pnp_ctx *ctx, uint64_t *d, uint64_t n, uint64_t seed) {
    if (!ctx || !d) return PNP_E_ARG;
    PNP_TRY(k_random_fr(d, n, seed, ctx->stream));
}

int pnp_synth_srs(pnp_ctx *ctx, uint64_t *d, uint64_t n, const uint64_t tau[4]) {
    if (!ctx || !d || !tau) return PNP_E_ARG;
    PNP_TRY(k_srs(d, n, from_u64_limbs<FrP>(tau), ctx->stream));
}

int pnp_synth_circuit(pnp_ctx *ctx, uint64_t *const w[4], uint64_t *const sel[9],
                      uint64_t *const sigma[4], uint64_t n, uint64_t n_gates, uint64_t pi_pos,
                      const uint64_t pi_canon[4]) {
    if (!ctx || !w || !sel || !sigma || !pi_canon || n_gates == 0 || n_gates > n || pi_pos >= n_gates)
        return PNP_E_ARG;
    PNP_TRY(k_synth_circuit(w, sel, sigma, n, n_gates, pi_pos, to_mont(from_u64_limbs<FrP>(pi_canon)),
                            ctx->stream));
}

int pnp_synth_merkle(pnp_ctx *ctx, uint32_t height, const uint64_t *consts, const uint64_t *d_leaves,
                     const uint64_t *d_blind, uint64_t *d_nodes, uint64_t *const w[4], uint64_t *const sel[9],
                     uint64_t *const sigma[4], uint64_t n, uint64_t root_canon[4]) {
    if (!ctx || !consts || !d_leaves || !d_blind || !d_nodes || !w || !sel || !sigma || !root_canon)
        return PNP_E_ARG;
    try {
        std::vector<uint64_t> pc(199 * 4);
        for (int k = 0; k < 199; k++) to_u64_limbs(to_mont(from_u64_limbs<FrP>(consts + 4 * k)), &pc[4 * k]);
        k_synth_merkle((int)height, pc.data(), d_leaves, d_blind, d_nodes, w, sel, sigma, n, ctx->stream);
        uint64_t r[4];
        PNP_HIP(hipMemcpy(r, d_nodes, 32, hipMemcpyDeviceToHost));
        to_u64_limbs(from_mont(from_u64_limbs<FrP>(r)), root_canon);
        return PNP_OK;
    } catch (const Error &e) {
        return e.code;
    }
}

int pnp_synth_coset_consts(pnp_ctx *ctx, uint64_t *d_vh, uint64_t *d_x, uint32_t lg_n) {
    if (!ctx || lg_n > 25) return PNP_E_ARG;
    PNP_TRY(k_coset_consts(d_vh, d_x, lg_n, ctx->stream));
}

}  // extern "C"

// ---------------------------------------------------------------- keys + prove
namespace {

enum FieldKind { kSkip, kEvals8, kCoeffs, kSelEvals8, kSelCoeffs, kTable };

// ProverKeyC field order (lib.rs:157-223) -> how gen_proof uses it.  The
// q_m, custom-gate and q_lookup selectors (kSel*) are read only when their 8n
// evaluations are non-zero: for the zero polynomial the Rust prover key holds
// EMPTY coefficient Vecs (prover.rs:765-808 passes their dangling pointers),
// so those coefficients are never touched.
const FieldKind kPkKinds[44] = {
    kSelCoeffs, kSelEvals8,                           // q_m
    kCoeffs, kEvals8, kCoeffs, kEvals8, kCoeffs, kEvals8, kCoeffs, kEvals8,  // q_l q_r q_o q_4
    kCoeffs, kEvals8, kCoeffs, kEvals8, kCoeffs, kEvals8, kCoeffs, kEvals8,  // q_c q_hl q_hr q_h4
    kCoeffs, kEvals8,                                 // q_arith
    kSelCoeffs, kSelEvals8, kSelCoeffs, kSelEvals8,   // range, logic selectors
    kSelCoeffs, kSelEvals8, kSelCoeffs, kSelEvals8,   // fixed / variable group add selectors
    kSelCoeffs, kSelEvals8,                           // q_lookup
    kTable, kTable, kTable, kTable,                   // table1..4 (n each, MultiSet::pad)
    kCoeffs, kEvals8, kCoeffs, kEvals8, kCoeffs, kEvals8, kCoeffs, kEvals8,  // sigmas
    kEvals8, kEvals8};                                // linear_evaluations, v_h_coset_8n
// selector fields (coefficients index; evaluations follow): q_m, range,
// logic, fixed group add, variable group add, q_lookup
const int kSelField[6] = {0, 20, 22, 24, 26, 28};

bool host_all_zero(const uint64_t *p, uint64_t words) {
    uint64_t acc = 0;
    for (uint64_t i = 0; i < words; i++) acc |= p[i];
    return acc == 0;
}

}  // namespace

extern "C" {

int pnp_load_prover_key(pnp_ctx *ctx, const ProverKeyC *pk, uint64_t D, int device_ptrs) {
    if (!ctx || !pk || D == 0 || (D & (D - 1)) || D > (1ULL << 25)) return PNP_E_ARG;
    PNP_TRY({
        tables_wait(ctx);  // a background build reads the key being replaced: let it finish
        PNP_HIP(hipSetDevice(ctx->device));
        ctx->pk_loaded = false;
        ctx->pk_gen++;  // derived groups (wires.hip) re-check sigma
        // device copies are kept across loads and reused when a field's size is
        // unchanged (the v1 symbol reloads every call: no hipMalloc / hipFree of
        // ~20 GiB per call)
        ctx->pk_owned.resize(44);
        ProverKeyC dev{};
        uint64_t *const *src = reinterpret_cast<uint64_t *const *>(pk);
        uint64_t **dst = reinterpret_cast<uint64_t **>(&dev);
        // non-zero selectors first: they decide which coefficient Vecs exist
        bool sel_nz[44] = {};
        for (int k = 0; k < 6; k++) {
            const int f = kSelField[k] + 1;
            if (!src[f]) {
                set_error("prover key field %d is null", f);
                throw Error(PNP_E_ARG);
            }
            const uint64_t words = 4 * 8 * D;
            const bool nz = device_ptrs ? pnp::k_any_nonzero(src[f], words, ctx->scratch_b, ctx->stream)
                                        : !host_all_zero(src[f], words);
            sel_nz[f] = sel_nz[f - 1] = nz;
        }
        std::vector<H2D> up;  // host fields, uploaded together (h2d_batch)
        for (int f = 0; f < 44; f++) {
            FieldKind k = kPkKinds[f];
            dst[f] = nullptr;
            if (k == kSkip || ((k == kSelEvals8 || k == kSelCoeffs) && !sel_nz[f])) {
                ctx->pk_owned[f].release();
                continue;
            }
            uint64_t elems = (k == kEvals8 || k == kSelEvals8) ? 8 * D : D;
            if (!src[f]) {
                set_error("prover key field %d is null", f);
                throw Error(PNP_E_ARG);
            }
            if (device_ptrs) {
                ctx->pk_owned[f].release();
                dst[f] = src[f];
            } else {
                auto &o = ctx->pk_owned[f];
                if (o.bytes != elems * 32) o.alloc(elems * 32);
                up.push_back({o.p, src[f], elems * 32});
                dst[f] = o.u64();
            }
        }
        h2d_batch(ctx, up);
        // key-derived constants, computed once per key instead of per proof:
        // zero-selector flags (the quotient kernel skips known-zero selectors)
        // and the sigma n-domain evaluations (gen_proof.cuh:159-165 recomputes
        // NTT.forward(sigma_coeffs) every proof)
        ctx->pk_qm_zero = dev.q_m_evals == nullptr;
        ctx->pk_qlookup_zero = dev.q_lookup_evals == nullptr;
        ctx->pk_custom_nz[0] = dev.range_selector_evals != nullptr;
        ctx->pk_custom_nz[1] = dev.logic_selector_evals != nullptr;
        ctx->pk_custom_nz[2] = dev.fixed_group_add_selector_evals != nullptr;
        ctx->pk_custom_nz[3] = dev.variable_group_add_selector_evals != nullptr;
        const uint64_t *sigc[4] = {dev.left_sigma_coeffs, dev.right_sigma_coeffs,
                                   dev.out_sigma_coeffs, dev.fourth_sigma_coeffs};
        uint32_t lg = 0;
        while ((1ULL << lg) < D) lg++;
        for (int j = 0; j < 4; j++) {
            if (ctx->pk_sigma_n[j].bytes < 32 * D) ctx->pk_sigma_n[j].alloc(32 * D);
            PNP_HIP(hipMemcpyAsync(ctx->pk_sigma_n[j].p, sigc[j], 32 * D, hipMemcpyDeviceToDevice,
                                   ctx->stream));
            pnp::ntt_run(ctx->ntt, ctx->pk_sigma_n[j].u64(), lg, false, false, ctx->stream);
        }
        // coset constants: v_h^-1 (the reference divides by v_h every proof,
        // quotient.cu:369-370); when the key's coset arrays are the standard
        // ones (x_i = 7 w_8n^i, v_h = x^n - 1, as every key built by the
        // reference's preprocessing), the L1 and PI coset evaluations have the
        // closed forms of protocol.h and need no LDE per proof
        const uint64_t N8 = 8 * D;
        auto tmp = [&](int k) -> pnp::DevBuf & {  // per-load scratch, kept for the next load
            if (ctx->pk_tmp[k].bytes != 32 * N8) ctx->pk_tmp[k].alloc(32 * N8);
            return ctx->pk_tmp[k];
        };
        pnp::DevBuf &vh_inv = tmp(0), &l1v = tmp(1);
        PNP_HIP(hipMemcpyAsync(vh_inv.p, dev.v_h_coset_8n, 32 * N8, hipMemcpyDeviceToDevice,
                               ctx->stream));
        pnp::k_batch_inverse(vh_inv.u64(), N8, ctx->scratch_a, ctx->stream);
        {
            pnp::DevBuf &vh = tmp(2), &x = tmp(3);
            pnp::k_coset_consts(vh.u64(), x.u64(), lg, ctx->stream);
            ctx->pk_std_coset =
                !pnp::k_any_diff(vh.u64(), dev.v_h_coset_8n, 4 * N8, ctx->scratch_b, ctx->stream) &&
                !pnp::k_any_diff(x.u64(), dev.linear_evaluations, 4 * N8, ctx->scratch_b, ctx->stream);
            if (ctx->pk_std_coset) {
                pnp::k_affine(l1v.u64(), x.u64(), Fr::one(), pnp::neg(Fr::one()), N8, ctx->stream);
                pnp::k_batch_inverse(l1v.u64(), N8, ctx->scratch_a, ctx->stream);
                Fr nf = Fr::zero();
                nf.v[0] = (uint32_t)D;
                nf.v[1] = (uint32_t)(D >> 32);
                pnp::k_affine(l1v.u64(), l1v.u64(), pnp::inverse(pnp::to_mont(nf)), Fr::zero(), N8,
                              ctx->stream);
            }
            PNP_HIP(hipStreamSynchronize(ctx->stream));
        }
        // The quotient's 8n arrays in block layout (point 8j + m -> block m,
        // index j), only the blocks this rank owns: all 8 on one GPU; 8/world
        // when the round-4 pipeline is distributed (pnp_set_exchange_a2a)
        const int world = ctx->msm.world;
        const bool split = world > 1 && 8 % world == 0 && ctx->msm.alltoall;
        ctx->pk_nb = split ? 8 / world : 8;
        ctx->pk_mb0 = split ? ctx->msm.rank * ctx->pk_nb : 0;
        // k_quotient29's keys (protocol.h): no custom gate, no lookup selector
        // or table, the standard coset; their selector / sigma / lin blocks are
        // kept in the 2^261 form (pk_blk29) and, but lin (the PI term), not in
        // the 2^256 form at all
        bool q29 = false;
        {
            static const bool q29_on = [] {
                const char *e = getenv("PNP_QUOT29");
                return !e || atoi(e) != 0;
            }();
            q29 = q29_on && ctx->pk_std_coset && ctx->pk_qlookup_zero && !ctx->pk_custom_nz[0] &&
                  !ctx->pk_custom_nz[1] && !ctx->pk_custom_nz[2] && !ctx->pk_custom_nz[3];
            const uint64_t *tabs[4] = {dev.table1, dev.table2, dev.table3, dev.table4};
            for (int k = 0; k < 4 && q29; k++)
                q29 = !tabs[k] || !pnp::k_any_nonzero(tabs[k], 4 * D, ctx->scratch_b, ctx->stream);
        }
        std::vector<std::string> used, used29;
        const uint64_t blk_elems = (uint64_t)ctx->pk_nb * D;
        auto put = [&](std::map<std::string, pnp::DevBuf> &m, std::vector<std::string> &u, const char *name,
                       const uint64_t *src, bool form29) {
            auto &b = m[name];
            if (b.bytes != 32 * blk_elems) b.alloc(32 * blk_elems);
            pnp::to_blocks(src, b.u64(), lg, ctx->pk_mb0, ctx->pk_nb, ctx->stream);
            if (form29) pnp::k_to_form29(b.u64(), b.u64(), blk_elems, ctx->stream);  // elementwise, in place
            u.push_back(name);
        };
        auto blk = [&](const char *name, const uint64_t *src) {
            static const char *const names29[] = {"q_m", "q_l", "q_r", "q_o", "q_4", "q_c", "q_hl", "q_hr",
                                                  "q_h4", "q_arith", "sig0", "sig1", "sig2", "sig3", "lin"};
            bool in29 = false;
            for (const char *nm : names29) in29 |= strcmp(nm, name) == 0;
            if (q29 && in29) put(ctx->pk_blk29, used29, name, src, true);
            if (!(q29 && in29) || strcmp(name, "lin") == 0) put(ctx->pk_blk, used, name, src, false);
        };
        if (!ctx->pk_qm_zero) blk("q_m", dev.q_m_evals);
        if (!ctx->pk_qlookup_zero) blk("q_lookup", dev.q_lookup_evals);
        if (ctx->pk_custom_nz[0]) blk("range", dev.range_selector_evals);
        if (ctx->pk_custom_nz[1]) blk("logic", dev.logic_selector_evals);
        if (ctx->pk_custom_nz[2]) blk("fixed_add", dev.fixed_group_add_selector_evals);
        if (ctx->pk_custom_nz[3]) blk("var_add", dev.variable_group_add_selector_evals);
        blk("q_l", dev.q_l_evals);
        blk("q_r", dev.q_r_evals);
        blk("q_o", dev.q_o_evals);
        blk("q_4", dev.q_4_evals);
        blk("q_c", dev.q_c_evals);
        blk("q_hl", dev.q_hl_evals);
        blk("q_hr", dev.q_hr_evals);
        blk("q_h4", dev.q_h4_evals);
        blk("q_arith", dev.q_arith_evals);
        blk("sig0", dev.left_sigma_evals);
        blk("sig1", dev.right_sigma_evals);
        blk("sig2", dev.out_sigma_evals);
        blk("sig3", dev.fourth_sigma_evals);
        blk("lin", dev.linear_evaluations);
        blk("vh_inv", vh_inv.u64());
        if (ctx->pk_std_coset) blk("l1v", l1v.u64());
        // blocks of an earlier key this one does not have
        auto prune = [](std::map<std::string, pnp::DevBuf> &m, const std::vector<std::string> &u) {
            for (auto it = m.begin(); it != m.end();)
                it = std::find(u.begin(), u.end(), it->first) == u.end() ? m.erase(it) : std::next(it);
        };
        prune(ctx->pk_blk, used);
        prune(ctx->pk_blk29, used29);
        ctx->pk_q29 = q29;
        // the coset-constant scratch (4 x 8n Fr) is kept only for callers that
        // load keys from host memory again and again (the v1 symbol); a
        // device-resident key is loaded once (and ranks sharing a GPU need the
        // HBM)
        if (device_ptrs) {
            PNP_HIP(hipStreamSynchronize(ctx->stream));
            for (auto &b : ctx->pk_tmp) b.release();
        }
        ctx->pk_blk_rank = ctx->msm.rank;
        ctx->pk_blk_world = world;
        ctx->pk_pinv.release();
        ctx->pk_pinv_pos = ~0ULL;
        PNP_HIP(hipStreamSynchronize(ctx->stream));
        ctx->pk_dev = dev;
        ctx->pk_n = D;
        ctx->pk_loaded = true;
        ctx->hbm_checked = false;  // the budget is checked by the next proof (pnp::hbm_budget)
    });
}

}  // extern "C"

namespace {

// make `up` (n_points packed affine points in HBM) the resident SRS.  The
// folded MSM table built from the previous SRS stays valid when the bytes are
// the same (a per-call upload of an unchanged key, as the v1 symbol does).
void adopt_ck(pnp_ctx *ctx, pnp::DevBuf &up, uint64_t n_points) {
    const bool same = ctx->ck_owned.p && ctx->ck_dev == ctx->ck_owned.u64() && ctx->ck_points == n_points &&
                      !pnp::k_any_diff(up.u64(), ctx->ck_owned.u64(), 12 * n_points, ctx->scratch_b, ctx->stream);
    PNP_HIP(hipStreamSynchronize(ctx->stream));
    if (!same) {
        std::swap(ctx->ck_owned, up);
        ctx->ck_dev = ctx->ck_owned.u64();
        pnp::ck_derived_reset(ctx);  // rebuilt from the new key on the next commitment
    }
    ctx->ck_points = n_points;
    ctx->ck_loaded = true;
    ctx->hbm_checked = false;
}

}  // namespace

extern "C" {

int pnp_load_commit_key(pnp_ctx *ctx, const CommitKeyC *ck, uint64_t n_points, int device_ptrs) {
    if (!ctx || !ck || !ck->powers_of_g || n_points == 0) return PNP_E_ARG;
    PNP_TRY({
        tables_wait(ctx);  // a background build reads the SRS being replaced: let it finish
        PNP_HIP(hipSetDevice(ctx->device));
        ctx->ck_loaded = false;
        if (device_ptrs) {
            // the tables derived from the SRS survive a reload of the same
            // bytes (same address, size and content hash)
            uint64_t h[2];
            pnp::k_hash_words(ck->powers_of_g, 12 * n_points, ctx->scratch_b, ctx->stream, h);
            const bool same = ctx->ck_hash_valid && !ctx->ck_owned.p && ctx->ck_dev == ck->powers_of_g &&
                              ctx->ck_points == n_points && h[0] == ctx->ck_hash[0] && h[1] == ctx->ck_hash[1];
            ctx->ck_owned.release();
            ctx->ck_dev = ck->powers_of_g;
            ctx->ck_points = n_points;
            if (!same) pnp::ck_derived_reset(ctx);
            ctx->ck_hash[0] = h[0];
            ctx->ck_hash[1] = h[1];
            ctx->ck_hash_valid = true;
            ctx->ck_loaded = true;
            ctx->hbm_checked = false;
        } else {
            ctx->ck_hash_valid = false;
            // upload (as the reference does per call, load.cu:348-358)
            pnp::DevBuf up(n_points * 96);
            h2d_batch(ctx, {{up.p, ck->powers_of_g, n_points * 96}});
            adopt_ck(ctx, up, n_points);
        }
    });
}

int pnp_load_commit_key_strided(pnp_ctx *ctx, const void *points, uint64_t n_points,
                                const pnp_affine_layout *layout, int device_ptrs) {
    if (!ctx || !points || !layout || n_points == 0) return PNP_E_ARG;
    const pnp_affine_layout L = *layout;
    if (L.stride % 8 || L.x_off % 8 || L.y_off % 8 || L.x_off + 48 > L.stride || L.y_off + 48 > L.stride ||
        L.inf_off >= L.stride || (L.x_off < L.y_off + 48 && L.y_off < L.x_off + 48) ||
        (L.inf_off >= L.x_off && L.inf_off < L.x_off + 48) || (L.inf_off >= L.y_off && L.inf_off < L.y_off + 48)) {
        pnp::set_error("affine layout: stride %llu, x at %llu, y at %llu, infinity at %llu is not a G1Affine layout",
                       (unsigned long long)L.stride, (unsigned long long)L.x_off, (unsigned long long)L.y_off,
                       (unsigned long long)L.inf_off);
        return PNP_E_ARG;
    }
    PNP_TRY({
        tables_wait(ctx);
        PNP_HIP(hipSetDevice(ctx->device));
        ctx->ck_loaded = false;
        pnp::DevBuf raw;
        const uint8_t *src = static_cast<const uint8_t *>(points);
        if (!device_ptrs) {
            raw.alloc(n_points * L.stride);
            PNP_HIP(hipMemcpyAsync(raw.p, points, n_points * L.stride, hipMemcpyHostToDevice, ctx->stream));
            src = static_cast<const uint8_t *>(raw.p);
        }
        pnp::DevBuf up(n_points * 96);
        if (!pnp::k_pack_affine(src, n_points, L.stride, L.x_off, L.y_off, L.inf_off, up.u64(), ctx->scratch_b,
                                ctx->stream)) {
            pnp::set_error("commit key holds the point at infinity (an SRS [tau^i] G never does)");
            throw pnp::Error(PNP_E_ARG);
        }
        raw.release();
        adopt_ck(ctx, up, n_points);
    });
}

uint32_t pnp_proof_infinity_mask(const ProofC *p) {
    if (!p) return 0;
    const CommitmentC *c = reinterpret_cast<const CommitmentC *>(p);
    uint64_t one[6];
    to_u64_limbs(Fq::one(), one);
    uint32_t m = 0;
    for (int k = 0; k < PNP_PROOF_COMMITMENTS; k++) {
        bool x0 = true;
        for (int j = 0; j < 6; j++) x0 &= c[k].x[j] == 0;
        if (x0 && !memcmp(c[k].y, one, 48)) m |= 1u << k;
    }
    return m;
}

int pnp_prove(pnp_ctx *ctx, const CircuitC *cs, int device_ptrs, ProofC *out) {
    if (!ctx || !cs || !out) return PNP_E_ARG;
    try {
        return prove_impl(ctx, cs, device_ptrs, out);
    } catch (const Error &e) {
        return e.code;
    } catch (const std::exception &e) {  // (bad_alloc, system_error: never across the C ABI)
        set_error("exception: %s", e.what());
        return PNP_E_DEVICE;
    } catch (...) {
        set_error("unknown exception");
        return PNP_E_DEVICE;
    }
}

int pnp_prove_ex(pnp_ctx *ctx, const CircuitC *cs, int device_ptrs, uint64_t n_pi, const uint64_t *pi_pos,
                 const uint64_t *pi_canon, const char *label, ProofC *out) {
    if (!ctx || !cs || !out || (n_pi && (!pi_pos || !pi_canon))) return PNP_E_ARG;
    ProveOpts o{n_pi, pi_pos, pi_canon, label ? label : "Merkle tree"};
    try {
        return prove_impl(ctx, cs, device_ptrs, out, &o);
    } catch (const Error &e) {
        return e.code;
    } catch (const std::exception &e) {
        set_error("exception: %s", e.what());
        return PNP_E_DEVICE;
    } catch (...) {
        set_error("unknown exception");
        return PNP_E_DEVICE;
    }
}

int pnp_last_stage_times(pnp_ctx *ctx, double *ms, const char **names, int cap) {
    if (!ctx) return 0;
    int k = 0;
    for (auto &st : ctx->stages) {
        if (k < cap) {
            if (ms) ms[k] = st.second;
            if (names) names[k] = st.first.c_str();
        }
        k++;
    }
    return k;
}

}  // extern "C"

namespace {

// v1 keys.  The reference copies every key array to the device on every call
// (load.cu:311-358, gen_proof.cuh:64-78, 166-180, 280-314: ~22 GiB at
// HEIGHT=15), so a caller may rewrite its key buffers in place between calls.
// The v1 symbol keeps that contract by default without the upload: every word
// the key load reads is hashed on the host (pk_content_hash / ck_content_hash
// below), and a key whose hash differs from the resident copy's is uploaded
// (pnp_load_*), so the proof always reads the caller's current key.  While
// both keys are resident, the hash runs beside the proof on the resident keys
// (speculation): equal hashes return that proof; a changed key is uploaded and
// the proof made again (PNP_V1_NO_SPECULATE=1: hash first, then prove).  The
// expensive objects derived from the SRS (the folded MSM tables, the Lagrange
// basis of lagrange.hip) are kept when an uploaded SRS equals the resident
// one byte for byte (compared on the device, pnp_load_commit_key).
// PNP_V1_RELOAD=1: upload both keys on every call (the reference's behaviour).
// PNP_V1_REUSE=1 (opt-in, for callers that never mutate their keys, like
// merkle-tree's main.rs and pnp_bench.rs): the resident copy made by an
// earlier call is reused while the key's fingerprint (every field pointer, the
// domain, and 257 evenly spaced words of every array the prover reads) is
// unchanged, saving the ~22 GiB upload.
// PNP_V1_STRICT=1: reject prover keys outside the reference GPU path's
// envelope (non-zero custom-gate selectors, q_lookup or lookup tables), for
// which this backend returns the ZK-Garage prover's proof while the reference
// GPU path would return a different one.
bool key_tables_zero(pnp_ctx *ctx) {
    const uint64_t *t[4] = {ctx->pk_dev.table1, ctx->pk_dev.table2, ctx->pk_dev.table3, ctx->pk_dev.table4};
    for (const uint64_t *p : t)
        if (p && pnp::k_any_nonzero(p, 4 * ctx->pk_n, ctx->scratch_b, ctx->stream)) return false;
    return true;
}
uint64_t mix64(uint64_t h, uint64_t v) {
    h ^= v + 0x9e3779b97f4a7c15ULL + (h << 6) + (h >> 2);
    return h * 0xff51afd7ed558ccdULL;
}
uint64_t sample_words(uint64_t h, const uint64_t *p, uint64_t words) {
    const uint64_t K = 256;
    for (uint64_t k = 0; k <= K; k++) h = mix64(h, p[(words - 1) * k / K]);
    return h;
}
uint64_t pk_fingerprint(const ProverKeyC &pk, uint64_t D) {
    uint64_t *const *f = reinterpret_cast<uint64_t *const *>(&pk);
    uint64_t h = mix64(0x1234567ULL, D);
    for (int i = 0; i < 44; i++) {
        h = mix64(h, reinterpret_cast<uintptr_t>(f[i]));
        FieldKind k = kPkKinds[i];
        // selector coefficients may be empty Vecs: pointer only (their
        // evaluations, sampled, decide whether they are read)
        if (k == kSkip || k == kSelCoeffs || !f[i]) continue;
        const uint64_t elems = (k == kEvals8 || k == kSelEvals8) ? 8 * D : D;
        h = sample_words(h, f[i], 4 * elems);
    }
    return h;
}
// Full-content key hash (the v1 default): every word of every array the key
// load reads, hashed on the host by up to 16 threads (memory-bound: ~17 GiB at
// HEIGHT=15 in ~0.1-0.2 s, against ~0.55 s to upload it over PCIe), so an
// unchanged key is not uploaded again while any change — in any word — is.
// Per 8 MiB chunk a 4-lane multiply-fold hash (two 64-bit digests of the four
// lane states) and the OR of its words (a selector's all-zero test), chunks
// combined in order.
struct Seg {
    const uint64_t *p;
    uint64_t words;
};
struct SegHash {
    uint64_t h0 = 0, h1 = 0;
    bool nz = false;
};
inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t mum(uint64_t a, uint64_t b) {  // 64 x 64 -> 128, folded (wyhash's mixer)
    const unsigned __int128 t = (unsigned __int128)a * b;
    return (uint64_t)t ^ (uint64_t)(t >> 64);
}
void hash_chunk(const uint64_t *p, uint64_t w, uint64_t seed, uint64_t out[3]) {
    // 4 independent lanes, one 128-bit product per word: ~1 word per cycle,
    // faster than host memory
    const uint64_t K[4] = {0xa0761d6478bd642fULL, 0xe7037ed1a0b428dbULL, 0x8ebc6af09c88c6e3ULL,
                           0x589965cc75374cc3ULL};
    uint64_t a[4] = {seed ^ K[0], seed ^ K[1], seed ^ K[2], seed ^ K[3]};
    uint64_t o = 0, i = 0;
    for (; i + 4 <= w; i += 4) {
        for (int k = 0; k < 4; k++) {
            const uint64_t v = p[i + k];
            o |= v;
            a[k] = mum(v ^ a[k], K[k]) ^ v;
        }
    }
    for (; i < w; i++) {
        o |= p[i];
        a[0] = mum(p[i] ^ a[0], K[0]) ^ p[i];
    }
    out[0] = mix64(mix64(mix64(mix64(w, a[0]), a[1]), a[2]), a[3]);
    out[1] = mum(a[0] ^ K[2], a[1] ^ K[3]) ^ mum(a[2] ^ K[0], a[3] ^ K[1]) ^ w;
    out[2] = o;
}
std::vector<SegHash> hash_segments(const std::vector<Seg> &segs, unsigned cap = 0) {
    const uint64_t CH = 1 << 20;  // words per chunk (8 MiB)
    struct Job {
        int seg;
        uint64_t off, w;
    };
    std::vector<Job> jobs;
    for (int k = 0; k < (int)segs.size(); k++)
        for (uint64_t o = 0; o < segs[k].words; o += CH) jobs.push_back({k, o, std::min(CH, segs[k].words - o)});
    std::vector<uint64_t> res(jobs.size() * 3);
    std::atomic<size_t> next{0};
    auto work = [&]() {
        for (size_t j; (j = next.fetch_add(1)) < jobs.size();)
            hash_chunk(segs[jobs[j].seg].p + jobs[j].off, jobs[j].w, jobs[j].off, &res[3 * j]);
    };
    unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (const char *e = getenv("OMP_NUM_THREADS")) T = std::max(1, std::min(atoi(e), 64));
    if (cap) T = std::min(T, cap);
    T = (unsigned)std::min<size_t>(T, std::max<size_t>(1, jobs.size()));
    std::vector<std::thread> th;
    try {
        for (unsigned t = 1; t < T; t++) th.emplace_back(work);
    } catch (...) {  // a thread that could not start: the started ones finish the jobs
    }
    work();
    for (auto &t : th) t.join();
    std::vector<SegHash> out(segs.size());
    for (size_t j = 0; j < jobs.size(); j++) {
        SegHash &h = out[jobs[j].seg];
        h.h0 = mix64(h.h0, res[3 * j]);
        h.h1 = mix64(h.h1, res[3 * j + 1]);
        h.nz |= res[3 * j + 2] != 0;
    }
    return out;
}
// the prover key as pnp_load_prover_key reads it at domain D: the fields it
// copies, the selector evaluations it tests, and a selector's coefficients
// only when its evaluations are non-zero (an all-zero selector's coefficient
// Vec is empty, lib.rs:157-223)
std::array<uint64_t, 2> pk_content_hash(const ProverKeyC &pk, uint64_t D, unsigned cap = 0) {
    uint64_t *const *f = reinterpret_cast<uint64_t *const *>(&pk);
    std::vector<Seg> segs;
    std::vector<int> field;
    for (int i = 0; i < 44; i++) {
        const FieldKind k = kPkKinds[i];
        if (k == kSkip || k == kSelCoeffs || !f[i]) continue;
        segs.push_back({f[i], 4 * ((k == kEvals8 || k == kSelEvals8) ? 8 * D : D)});
        field.push_back(i);
    }
    std::vector<SegHash> h = hash_segments(segs, cap);
    std::vector<Seg> sel;
    for (size_t j = 0; j < segs.size(); j++)
        if (kPkKinds[field[j]] == kSelEvals8 && h[j].nz && f[field[j] - 1]) sel.push_back({f[field[j] - 1], 4 * D});
    std::vector<SegHash> hs = hash_segments(sel, cap);
    std::array<uint64_t, 2> r = {mix64(0xABCDEFULL, D), mix64(0xFEDCBAULL, D)};
    for (size_t j = 0; j < h.size(); j++) {
        r[0] = mix64(mix64(r[0], field[j]), h[j].h0);
        r[1] = mix64(mix64(r[1], field[j]), h[j].h1);
    }
    for (const SegHash &x : hs) r[0] = mix64(r[0], x.h0), r[1] = mix64(r[1], x.h1);
    return r;
}
std::array<uint64_t, 2> ck_content_hash(const CommitKeyC &ck, uint64_t D, unsigned cap = 0) {
    std::vector<SegHash> h = hash_segments({{ck.powers_of_g, 12 * D}}, cap);
    return {mix64(0x13579BULL ^ D, h[0].h0), mix64(0x2468ACULL ^ D, h[0].h1)};
}

uint64_t ck_fingerprint(const CommitKeyC &ck, uint64_t D) {
    uint64_t h = mix64(mix64(0x7654321ULL, D), reinterpret_cast<uintptr_t>(ck.powers_of_g));
    return ck.powers_of_g ? sample_words(h, ck.powers_of_g, 12 * D) : h;
}

}  // namespace

// The folded MSM table of a freshly uploaded SRS (what a context's first proof
// builds first: ~0.19 s at 2^22) built on a stream of its own, from a thread of
// its own (msm_build_table synchronises its stream and frees its level
// buffers), while the caller uploads the prover key over PCIe — the v1 cold
// call.  The first proof finds it (commit_table); if it could not be built
// (e.g. out of HBM) the proof builds it as before.  One GPU: the whole table.
static std::thread table_prebuild(pnp_ctx *ctx, uint64_t n) {
    return std::thread([ctx, n] {
        hipStream_t s = nullptr;
        try {
            PNP_HIP(hipSetDevice(ctx->device));
            PNP_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            ctx->ck_table_n = 0;
            msm_build_table(ctx->ck_table, ctx->ck_dev, n, ctx->msm.fold_c, s);
            ctx->ck_table_p0 = 0;
            ctx->ck_table_p1 = n;
            ctx->ck_table_n = n;
        } catch (...) {
            ctx->ck_table_n = 0;
        }
        if (s) (void)hipStreamDestroy(s);
    });
}

extern "C" {

// v1: lib/hello.cu:4-6.  Same contract as the reference (structs by value,
// synchronous, device 0, keys uploaded per call, print-and-exit on errors,
// caffe/common.hpp:23-30); see the v1 keys note above for the switches.
static pnp_ctx *g_v1_ctx = nullptr;  // the v1 symbol's context (pnp_v1_context)
pnp_ctx *pnp_v1_context(void) { return g_v1_ctx; }

ProofC gen_proof(CircuitC circuit, ProverKeyC pk, CommitKeyC ck) {
    pnp_ctx *&ctx = g_v1_ctx;
    static bool have_pk = false, have_ck = false;
    static std::array<uint64_t, 2> h_pk{}, h_ck{};
    auto env_on = [](const char *name) {  // read per call: a caller may switch modes
        const char *e = getenv(name);
        return e && atoi(e) != 0;
    };
    const bool reuse = env_on("PNP_V1_REUSE"), reload = env_on("PNP_V1_RELOAD"), strict = env_on("PNP_V1_STRICT");
    ProofC out;
    memset(&out, 0, sizeof out);
    auto die = [](int rc) {
        fprintf(stderr, "gen_proof: error %d: %s\n", rc, pnp_last_error());
        exit(EXIT_FAILURE);
    };
    int rc;
    // the cold call's own stages (HIP init + context, key uploads, the hasher's
    // tail after the proof), put before the proof's stages in
    // pnp_last_stage_times(pnp_v1_context()) — bench.py's process-cold line
    using clk = std::chrono::steady_clock;
    const auto t_call = clk::now();
    auto ms_since = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
    const bool cold_ctx = !ctx;
    if (!ctx && (rc = pnp_ctx_create(0, &ctx)) != PNP_OK) die(rc);
    const double ms_ctx = cold_ctx ? ms_since(t_call) : 0.0;
    uint64_t bound = circuit.n > circuit.lookup_len ? circuit.n : circuit.lookup_len;
    uint64_t D = 1;
    while (D < bound) D <<= 1;
    if (!ck.powers_of_g) die(PNP_E_ARG);
    // what identifies "the same key": the full-content hash (default), the
    // sampled fingerprint (PNP_V1_REUSE), nothing (PNP_V1_RELOAD: upload always)
    std::array<uint64_t, 2> hp{}, hc{};
    const bool speculate = !reuse && !reload && have_pk && have_ck && ctx->pk_loaded && ctx->ck_loaded &&
                           ctx->pk_n == D && ctx->ck_points == D && !env_on("PNP_V1_NO_SPECULATE");
    if (speculate) {
        // hash on the other cores (one fewer than the hash would take alone:
        // this thread drives the proof) while the proof runs on the resident keys
        unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        if (const char *e = getenv("OMP_NUM_THREADS")) T = std::max(1, std::min(atoi(e), 64));
        const unsigned cap = T > 1 ? T - 1 : 1;
        bool hash_ok = true;
        std::thread hasher([&] {
            try {
                hp = pk_content_hash(pk, D, cap);
                hc = ck_content_hash(ck, D, cap);
            } catch (...) {
                hash_ok = false;
            }
        });
        int prc;
        try {  // (pnp_prove returns codes; the join must happen whatever it does)
            prc = pnp_prove(ctx, &circuit, 0, &out);
        } catch (...) {
            hasher.join();
            throw;
        }
        hasher.join();
        if (hash_ok && hp == h_pk && hc == h_ck) {
            if (prc != PNP_OK) die(prc);
            return out;
        }
        // a changed key (or no hash): that proof read the old one; upload and prove again
        memset(&out, 0, sizeof out);
        if (!hash_ok) have_pk = have_ck = false;
    } else if (reuse) {
        hp = {pk_fingerprint(pk, D), D};
        hc = {ck_fingerprint(ck, D), D};
    } else if (!reload) {
        const bool load_pk = !have_pk || !ctx->pk_loaded || ctx->pk_n != D;
        const bool load_ck = !have_ck || !ctx->ck_loaded || ctx->ck_points != D;
        if (load_pk && load_ck) {
            // both keys are uploaded whatever their hashes (a cold call: the
            // reference driver's one proof per process): hash them on the
            // other cores beside the uploads and the proof, for the next call
            // (leaving this thread and the upload's copy threads their cores)
            unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
            if (const char *e = getenv("OMP_NUM_THREADS")) T = std::max(1, std::min(atoi(e), 64));
            const unsigned busy = 1 + pnp_ctx::kStgThreads;
            const unsigned cap = T > busy + 1 ? T - busy : 1;
            bool hash_ok = true;
            std::array<uint64_t, 2> ahp{}, ahc{};
            std::thread hasher([&] {
                try {
                    ahp = pk_content_hash(pk, D, cap);
                    ahc = ck_content_hash(ck, D, cap);
                } catch (...) {
                    hash_ok = false;
                }
            });
            int lrc = PNP_OK;
            bool envelope = true;
            double ms_pk = 0, ms_ck = 0, ms_prove = 0;
            std::thread tb;
            try {
                // the SRS first: its folded table builds on the GPU (table_prebuild)
                // while the prover key crosses PCIe
                auto t = clk::now();
                if ((lrc = pnp_load_commit_key(ctx, &ck, D, 0)) == PNP_OK) {
                    ms_ck = ms_since(t);
                    if (ctx->msm.world <= 1 && ctx->ck_table_n != D) tb = table_prebuild(ctx, D);
                    t = clk::now();
                    lrc = pnp_load_prover_key(ctx, &pk, D, 0);
                    if (tb.joinable()) tb.join();
                    if (lrc == PNP_OK) {
                        envelope = !strict || (ctx->pk_qm_zero && ctx->pk_qlookup_zero && !ctx->pk_custom_nz[0] &&
                                               !ctx->pk_custom_nz[1] && !ctx->pk_custom_nz[2] &&
                                               !ctx->pk_custom_nz[3] && key_tables_zero(ctx));
                        ms_pk = ms_since(t);
                        t = clk::now();
                        if (envelope) lrc = pnp_prove(ctx, &circuit, 0, &out);
                        ms_prove = ms_since(t);
                    }
                }
            } catch (...) {
                if (tb.joinable()) tb.join();
                hasher.join();
                throw;
            }
            const auto t_join = clk::now();
            hasher.join();
            {
                std::vector<std::pair<std::string, double>> st = {
                    {"v1_ctx_create", ms_ctx}, {"v1_load_prover_key", ms_pk}, {"v1_load_commit_key", ms_ck},
                    {"v1_prove", ms_prove}};
                st.insert(st.end(), ctx->stages.begin(), ctx->stages.end());
                st.push_back({"v1_hash_wait", ms_since(t_join)});
                st.push_back({"v1_call", ms_since(t_call)});
                ctx->stages.swap(st);
            }
            have_pk = have_ck = false;
            if (lrc != PNP_OK) die(lrc);
            if (!envelope) {
                set_error("PNP_V1_STRICT: prover key outside the reference GPU path's envelope (custom-gate "
                          "selectors, q_m, q_lookup or lookup tables non-zero)");
                die(PNP_E_ENVELOPE);
            }
            if (hash_ok) {  // (otherwise the next call uploads again)
                have_pk = have_ck = true;
                h_pk = ahp;
                h_ck = ahc;
            }
            return out;
        }
        hp = pk_content_hash(pk, D);
        hc = ck_content_hash(ck, D);
    }
    if (reload || !have_pk || hp != h_pk || !ctx->pk_loaded || ctx->pk_n != D) {
        have_pk = false;
        if ((rc = pnp_load_prover_key(ctx, &pk, D, 0)) != PNP_OK) die(rc);
        if (strict && (!ctx->pk_qm_zero || !ctx->pk_qlookup_zero || ctx->pk_custom_nz[0] ||
                       ctx->pk_custom_nz[1] || ctx->pk_custom_nz[2] || ctx->pk_custom_nz[3] ||
                       !key_tables_zero(ctx))) {
            set_error("PNP_V1_STRICT: prover key outside the reference GPU path's envelope (custom-gate "
                      "selectors, q_m, q_lookup or lookup tables non-zero)");
            die(PNP_E_ENVELOPE);
        }
        have_pk = true;
        h_pk = hp;
    }
    if (reload || !have_ck || hc != h_ck || !ctx->ck_loaded || ctx->ck_points != D) {
        have_ck = false;
        if ((rc = pnp_load_commit_key(ctx, &ck, D, 0)) != PNP_OK) die(rc);
        have_ck = true;
        h_ck = hc;
    }
    if ((rc = pnp_prove(ctx, &circuit, 0, &out)) != PNP_OK) die(rc);
    return out;
}

}  // extern "C"
