// msm.hip — Pippenger MSM on BLS12-381 G1 for gfx950.
//
// Contract of the reference's multi_scalar_mult (utils/function.cu:275-290 ->
// zksnark_msm.cu:45-83 -> sppark_msm/pippenger.cuh:470-556, CPU fold in
// zkp/cpu/collect.h:326-489): sum_i s_i * P_i for n affine Montgomery points
// and n scalars (here Montgomery in, canonicalised on the device, as
// to_base in PLONK/src/arithmetic.cu:3-8).
//
// Two layouts of the same pipeline:
//   * per-window (arbitrary points, pnp_commit): every c-bit window of every
//     MSM owns NB = 2^(c-1) buckets; window sums meet in a host Horner step.
//   * folded (the resident SRS, every gen_proof commitment): the commit key is
//     expanded once into a table T[k*n + i] = 2^(c*k) P_i (W*n affine points,
//     6 GiB at n = 2^22 — HBM is 288 GB), so digit k of scalar i is a signed
//     multiple of T[k*n + i] and ALL windows of an MSM share one set of NB
//     buckets.  Same number of mixed additions, but the bucket reduction is W
//     times smaller and the result needs no doublings on the host.
//
// MI355X design (no cooperative kernels, no CPU bucket fold):
//   1. k_digits         : signed c-bit digits, |d| <= 2^(c-1), one u16 key per
//                         (window, point) — u32 key = (|d|-1) | sign<<31,
//                         KEY_ZERO for d = 0.
//   2. k_hist           : one workgroup per (virtual window, chunk of points)
//                         builds the chunk's bucket histogram in LDS (2^(c-1)
//                         u32 <= 128 KiB) over all the key rows of its virtual
//                         window, stored bucket-major, chunk-minor.
//   3. scan             : exclusive scan of those counts = the start of every
//                         (window, bucket, chunk) run in the sorted entry list.
//   4. k_scatter        : same workgroups place entries with LDS cursors — no
//                         global atomics anywhere.
//   5. accumulate       : XYZZ mixed additions (8M + 2S), k_accumulate_flat:
//                         every lane sums exactly S consecutive sorted entries
//                         across bucket boundaries; msm_merge_pieces joins the
//                         pieces of split buckets (msm_reduce.hip).
//   6. msm_reduce       : sum_b (b+1) B_b per virtual window (msm_reduce.hip).
//   7. host             : per-window layout: Horner over the windows; both:
//                         sum of the ranks' partial results, affine.
#include <algorithm>
#include "msm_internal.h"
#include "ec.cuh"
#include "ec29.cuh"

namespace pnp {

// ---------------------------------------------------------------- 1. digits
constexpr uint32_t KEY_ZERO = 0xFFFFFFFFu;
// the W signed c-bit digits of scalar i as keys (magnitude - 1 | sign << 31,
// KEY_ZERO for a zero digit), row w of keys at keys[w n + i]; fn(key) per digit
// top_sh (folded tables, MsmCfg::top_sh): the top window's digit d becomes
// magnitude d 2^top_sh (its table level is divided by 2^top_sh)
// C > 0: the window width known at compile time (c = 20, every folded MSM
// from 2^19 points): the limb index and shift of every window fold to
// constants, no selects (~20 VALU per digit less)
template <int C, class E>
__device__ __forceinline__ void digits_of(const Fr &s, int c_rt, int W_rt, int top_sh, E emit) {
    const int c = C > 0 ? C : c_rt;
    const int W = C > 0 ? (255 + C) / C : W_rt;
    const uint32_t NB = 1u << (c - 1);
    uint32_t carry = 0;
    auto digit = [&](int w) {
        const int bit = w * c;
        const int li = bit >> 5, sh = bit & 31;
        // limbs li, li + 1 by selects (a dynamic register index would go to scratch)
        uint32_t lo32 = 0, hi32 = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            lo32 = li == k ? s.v[k] : lo32;
            hi32 = li + 1 == k ? s.v[k] : hi32;
        }
        const uint64_t word = lo32 | ((uint64_t)hi32 << 32);
        uint32_t raw = (uint32_t)(word >> sh) & ((1u << c) - 1);
        raw += carry;
        uint32_t key = KEY_ZERO;
        if (raw > NB) {
            const uint32_t mag = (NB << 1) - raw;  // |raw - 2^c|, 0 when raw = 2^c
            carry = 1;
            if (mag) key = (mag - 1) | 0x80000000u;
        } else {
            carry = 0;
            if (raw) key = (w == W - 1 ? raw << top_sh : raw) - 1;
        }
        // the top window never carries: W c >= 255 + 1 for the configured c (scalars < 2^255)
        emit(w, key);
    };
    if constexpr (C > 0) {
#pragma unroll
        for (int w = 0; w < (255 + C) / C; w++) digit(w);
    } else {
        for (int w = 0; w < W; w++) digit(w);
    }
}
template <class F>
__device__ __forceinline__ void scalar_digits(const uint64_t *scalars, uint64_t i, uint64_t n, int c, int W,
                                              int top_sh, uint32_t *keys, F fn) {
    const Fr s = from_mont(load_fr(scalars, i));
    auto emit = [&](int w, uint32_t key) {
        keys[(uint64_t)w * n + i] = key;
        fn(key);
    };
    if (c == 20 && W == 13)
        digits_of<20>(s, c, W, top_sh, emit);
    else
        digits_of<0>(s, c, W, top_sh, emit);
}
__global__ void k_digits(const uint64_t *scalars, uint64_t n, int c, int W, int top_sh, uint32_t *keys) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    scalar_digits(scalars, i, n, c, W, top_sh, keys, [](uint32_t) {});
}

// Virtual window v reads `rows` key rows starting at row v*vstride + off of
// the key matrix (row r = keys[r*n .. r*n + n)); the entry of point i in its
// row j is  i + (id_row0 + j) * id_mul  (id_mul = 0: the point index itself;
// id_mul = n: the index into the folded table).
constexpr int MSM_BATCH_MAX = 16;  // MSMs per batch with per-MSM pointers / offsets
struct KeyRows {
    uint64_t n;
    int vstride, off, rows;
    uint32_t id_row0;
    uint64_t id_mul;
    uint64_t id_base = 0;  // added to every entry id (a rank's first point in the full folded table)
    // folded tables holding several point sets (MsmSegs): MSM v < nseg starts
    // at seg_off[v] of every table row (nseg = 0: one point set; the
    // per-window layout has more virtual windows than slots here)
    int nseg = 0;
    uint64_t seg_off[MSM_BATCH_MAX] = {};
};

// ---------------------------------------------------------------- 2. coarse pass
// Two-pass bucket sort.  Pass A sorts the entries by the top CB = 9 bits of
// the bucket (NBc = 512 coarse bins), pass B sorts each coarse bin by the
// remaining FB bits in one workgroup (folded c = 20 at 2^22: 2^19 buckets =
// 512 bins x 1024 fine bins, ~13 x 2^22 / 512 = 106K entries per coarse bin,
// ~104 per bucket).  Few bins keep the write fronts few; pass A also
// counting-sorts 4096-key tiles in LDS so each bin's entries leave as one run
// (a one-pass scatter straight to 2^15 buckets wrote ~8x its payload to HBM).
// Keys, fine keys and entries are read four per lane (8 / 4 / 16-byte loads).
#ifndef PNP_SORT_CB
#define PNP_SORT_CB 9
#endif
constexpr int SORT_CB = PNP_SORT_CB;
constexpr int SORT_FB_MAX = 11;
// three 2^CB-entry u32 LDS arrays + the 2 x 16 KiB tile of k_coarse_scatter
static_assert(SORT_CB >= 1 && SORT_CB <= 12, "PNP_SORT_CB out of range (LDS budget of k_coarse_scatter)");
// counts / offsets index of (virtual window v, coarse bin b, chunk ch):
// v-major; or, with wmaj > 1 destinations (bucket-range sharding: the top
// log2(wmaj) bits of b name the rank owning the bucket), destination-major,
// so every destination's entries are one contiguous run
__device__ __forceinline__ uint64_t cidx(int v, int nv, uint32_t b, int NBc, int wmaj, int ch, int nch) {
    if (wmaj <= 1) return ((uint64_t)v * NBc + b) * nch + ch;
    const uint32_t nbl = (uint32_t)NBc / wmaj;
    return (((uint64_t)(b / nbl) * nv + v) * nbl + b % nbl) * nch + ch;
}

__global__ __launch_bounds__(1024) void k_coarse_hist(const uint32_t *keys, KeyRows kr, int fb,
                                                      int NBc, uint64_t chunk, int nch,
                                                      uint32_t *counts, int wmaj = 1) {
    __shared__ uint32_t hist[1 << SORT_CB];
    const int v = blockIdx.y, ch = blockIdx.x;
    for (int b = threadIdx.x; b < NBc; b += blockDim.x) hist[b] = 0;
    __syncthreads();
    const uint64_t n = kr.n;
    uint64_t lo = (uint64_t)ch * chunk, hi = lo + chunk < n ? lo + chunk : n;
    const uint32_t *kb = keys + ((uint64_t)v * kr.vstride + kr.off) * n;
    const bool vec = ((n | chunk) & 3) == 0;  // four keys per 16-byte load
    for (int r = 0; r < kr.rows; r++) {
        const uint32_t *k = kb + (uint64_t)r * n;
        if (vec) {
            for (uint64_t i = lo + 4 * threadIdx.x; i < hi; i += 4 * blockDim.x) {
                uint4 q = *reinterpret_cast<const uint4 *>(k + i);
                uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (w[j] != KEY_ZERO) atomicAdd(&hist[(w[j] & 0x7FFFFFFFu) >> fb], 1u);
            }
        } else {
            for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
                uint32_t key = k[i];
                if (key != KEY_ZERO) atomicAdd(&hist[(key & 0x7FFFFFFFu) >> fb], 1u);
            }
        }
    }
    __syncthreads();
    for (int b = threadIdx.x; b < NBc; b += blockDim.x) counts[cidx(v, gridDim.y, b, NBc, wmaj, ch, nch)] = hist[b];
}

// k_digits + k_coarse_hist in one pass for the standard folded layout (every
// window of MSM v = blockIdx.y, keys of MSM v at keys + v W n): the keys are
// counted as they are made instead of being read back
struct ScalarPtrs {
    static constexpr int MAX = MSM_BATCH_MAX;
    const uint64_t *p[MAX];
};
__global__ __launch_bounds__(1024) void k_digits_hist(ScalarPtrs sp, uint64_t n, int c, int W, int top_sh, int fb,
                                                      int NBc,
                                                      uint64_t chunk, int nch, uint32_t *keys, uint32_t *counts,
                                                      int wmaj = 1) {
    __shared__ uint32_t hist[1 << SORT_CB];
    const int v = blockIdx.y, ch = blockIdx.x;
    for (int b = threadIdx.x; b < NBc; b += blockDim.x) hist[b] = 0;
    __syncthreads();
    const uint64_t lo = (uint64_t)ch * chunk, hi = lo + chunk < n ? lo + chunk : n;
    uint32_t *kv = keys + (uint64_t)v * W * n;
    for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x)
        scalar_digits(sp.p[v], i, n, c, W, top_sh, kv, [&](uint32_t key) {
            if (key != KEY_ZERO) atomicAdd(&hist[(key & 0x7FFFFFFFu) >> fb], 1u);
        });
    __syncthreads();
    for (int b = threadIdx.x; b < NBc; b += blockDim.x) counts[cidx(v, gridDim.y, b, NBc, wmaj, ch, nch)] = hist[b];
}

// ---------------------------------------------------------------- 3. scan
// exclusive scan of u32 in place, three phases over 1024-element tiles
__global__ __launch_bounds__(256) void k_scan_tiles(uint32_t *d, uint64_t n, uint32_t *tile_sums) {
    __shared__ uint32_t wsum[4];
    uint64_t base = (uint64_t)blockIdx.x * 1024;
    uint32_t v[4], loc = 0;
    for (int k = 0; k < 4; k++) {
        uint64_t i = base + threadIdx.x * 4 + k;
        v[k] = i < n ? d[i] : 0;
        loc += v[k];
    }
    // wave-level inclusive scan of loc
    uint32_t x = loc;
    int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    uint32_t wpre = 0;
    for (int j = 0; j < wv; j++) wpre += wsum[j];
    uint32_t excl = wpre + x - loc;
    for (int k = 0; k < 4; k++) {
        uint64_t i = base + threadIdx.x * 4 + k;
        if (i < n) d[i] = excl;
        excl += v[k];
    }
    if (threadIdx.x == 255) tile_sums[blockIdx.x] = wpre + x;
}
__global__ void k_scan_add(uint32_t *d, uint64_t n, const uint32_t *tile_pre) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < n) d[i] += tile_pre[i >> 10];
}
static void scan_u32(uint32_t *d, uint64_t n, DevBuf &scratch, hipStream_t s) {
    // recursive tile scan; scratch holds the per-level tile sums
    std::vector<std::pair<uint32_t *, uint64_t>> levels;
    uint64_t need = 0, m = n;
    while (m > 1) { m = (m + 1023) / 1024; need += m; }
    if (scratch.bytes < (need + 1) * 4) scratch.alloc((need + 1) * 4);
    uint32_t *p = static_cast<uint32_t *>(scratch.p);
    uint32_t *cur = d;
    m = n;
    while (true) {
        uint64_t tiles = (m + 1023) / 1024;
        hipLaunchKernelGGL(k_scan_tiles, dim3((uint32_t)tiles), dim3(256), 0, s, cur, m, p);
        PNP_HIP(hipGetLastError());
        levels.push_back({cur, m});
        if (tiles == 1) break;
        cur = p;
        p += tiles;
        m = tiles;
    }
    // propagate tile prefixes downwards
    for (int l = (int)levels.size() - 2; l >= 0; l--) {
        uint32_t *dd = levels[l].first;
        uint64_t mm = levels[l].second;
        uint32_t *pre = levels[l + 1].first;
        hipLaunchKernelGGL(k_scan_add, dim3((uint32_t)((mm + 255) / 256)), dim3(256), 0, s, dd, mm, pre);
        PNP_HIP(hipGetLastError());
    }
}

// ---------------------------------------------------------------- 4. scatters
// pass A: entry (table index | sign << 31) and its fine key, grouped by coarse
// bin.  Tiles of 16384 keys are counting-sorted in LDS first, so each bin's
// entries of a tile leave as one contiguous run (coalesced stores: ~32
// entries per bin and tile; 4096-key tiles left ~8-entry runs, and pass A took
// 3.9 instead of 3.3 ms per proof, A/B 0.1437 -> 0.1425 s per proof,
// profiles/r03_ab_sort_tiles.txt; one workgroup per CU with 134 KB of LDS).
#ifndef PNP_TILE_K
#define PNP_TILE_K 16384
#endif
// the next tile's loads issued before this tile's LDS phases (both passes)
#ifndef PNP_SORT_PREFETCH
#define PNP_SORT_PREFETCH 1
#endif
constexpr int TILE_K = PNP_TILE_K;
constexpr int KPT = TILE_K / 1024;  // keys per lane per tile
static_assert(TILE_K % 4096 == 0 && TILE_K <= 16384, "PNP_TILE_K: a multiple of 4096 up to 16384");
// exclusive scan of lh[0..nb) into lofs by the whole workgroup: each lane
// sums its run of ceil(nb / blockDim) bins, one wave-level scan, the wave
// totals through LDS (wsum: blockDim / 64 words).  Every lane must call it; the
// caller synchronises after it.  (PNP_SORT_SCAN=0: wave 0 alone, 32 bins per
// lane in sequence at 2048 fine bins while 15 waves wait at the barrier)
// (PNP_SORT_SCAN=1: the wave scan by __shfl_up, ds_bpermute through the LDS
// crossbar, and the wave totals summed one LDS read after another; 2: DPP
// row shifts / broadcasts in the VALU, and the totals of the <= 16 waves read
// once per lane and scanned the same way)
#ifndef PNP_SORT_SCAN
#define PNP_SORT_SCAN 2
#endif
// inclusive scan over the 64 lanes of a wave by DPP: row_shr 1, 2, 4, 8 inside
// each row of 16 lanes, then row_bcast:15 and row_bcast:31 carry the row totals
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x) {
    const uint32_t lane = threadIdx.x & 63, rl = lane & 15;
    uint32_t t = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    if (rl >= 1) x += t;
    t = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    if (rl >= 2) x += t;
    t = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    if (rl >= 4) x += t;
    t = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    if (rl >= 8) x += t;
    t = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x142, 0xf, 0xf, false);  // row_bcast:15
    if ((lane & 31) >= 16) x += t;
    t = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x143, 0xf, 0xf, false);  // row_bcast:31
    if (lane >= 32) x += t;
    return x;
}
__device__ __forceinline__ void tile_scan_wave0(uint32_t *lh, uint32_t *lofs, int nb);
__device__ __forceinline__ void tile_scan(uint32_t *lh, uint32_t *lofs, int nb, uint32_t *wsum) {
#if PNP_SORT_SCAN
    const int per = (nb + (int)blockDim.x - 1) / (int)blockDim.x, b0 = (int)threadIdx.x * per;
    uint32_t loc = 0;
    for (int b = b0; b < b0 + per && b < nb; b++) loc += lh[b];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#if PNP_SORT_SCAN == 2
    const uint32_t x = wave_scan_incl(loc);
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    // the waves before this one: every lane reads one wave total, one more scan
    const int nw = (int)blockDim.x >> 6;
    const uint32_t wt = wave_scan_incl(lane < nw ? wsum[lane] : 0u);
    const int wsrc = __builtin_amdgcn_readfirstlane(wv) - 1;
    uint32_t run = x - loc + (wsrc >= 0 ? (uint32_t)__builtin_amdgcn_readlane((int)wt, wsrc) : 0u);
#else
    uint32_t x = loc;
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    uint32_t run = x - loc;
    for (int j = 0; j < wv; j++) run += wsum[j];
#endif
    for (int b = b0; b < b0 + per && b < nb; b++) {
        lofs[b] = run;
        run += lh[b];
    }
#else
    (void)wsum;
    tile_scan_wave0(lh, lofs, nb);
#endif
}
__device__ __forceinline__ void tile_scan_wave0(uint32_t *lh, uint32_t *lofs, int nb) {
    // exclusive scan of lh[0..nb) into lofs by wave 0
    if (threadIdx.x < 64) {
        const int per = (nb + 63) / 64, b0 = threadIdx.x * per;
        uint32_t loc = 0;
        for (int b = b0; b < b0 + per && b < nb; b++) loc += lh[b];
        uint32_t x = loc;
        for (int off = 1; off < 64; off <<= 1) {
            uint32_t y = __shfl_up(x, off, 64);
            if ((int)threadIdx.x >= off) x += y;
        }
        uint32_t run = x - loc;
        for (int b = b0; b < b0 + per && b < nb; b++) {
            lofs[b] = run;
            run += lh[b];
        }
    }
}

// Tile ranking of pass A.  PNP_SORT_WAVERANK=0: one LDS atomic-with-return per
// key on the tile's bin counters.  1: wave-level ranking —
// each wave keeps its own 16-bit bin counters; a key's peers in its wave (same
// bin) come from one ballot per bin bit (match-any), its rank is the popcount of
// the peers below it (mbcnt), and the lowest peer alone adds the group to the
// wave's counter (a plain LDS read and write: a wave's LDS operations execute in
// order, so no atomic); the tile's bin offsets are then one scan over
// (bin, wave) in bin-major order, which also makes the tile's order stable
#ifndef PNP_SORT_WAVERANK
#define PNP_SORT_WAVERANK 0
#endif
constexpr int SORT_NW = 16;  // waves of a 1024-lane sort workgroup

// rec != nullptr: entries leave as 8-byte records entry | fine key << 32 (the
// bucket-range exchange format) instead of the ent / fk arrays.  slot_recs > 0
// (fixed-slot exchange): destination d's records go to its slot, rec + d
// slot_recs + hdr_recs, at most `cap` of them (the rest are dropped; the slot
// header, k_slot_header, flags the overflow and the batch is redone)
__global__ __launch_bounds__(1024) void k_coarse_scatter(const uint32_t *keys, KeyRows kr, int fb,
                                                         int NBc, uint64_t chunk, int nch,
                                                         const uint32_t *offs, uint32_t *ent,
                                                         uint16_t *fk, int wmaj = 1, uint64_t *rec = nullptr,
                                                         uint32_t slot_recs = 0, uint32_t hdr_recs = 0,
                                                         uint32_t cap = 0) {
    __shared__ uint32_t cur[1 << SORT_CB], lh[1 << SORT_CB], lofs[1 << SORT_CB], lim[1 << SORT_CB], wsum[16];
    __shared__ uint32_t st_e[TILE_K];
    __shared__ uint32_t st_m[TILE_K];
#if PNP_SORT_WAVERANK
    // per-wave bin counters (<= KPT * 64 per wave), then the (bin, wave) offsets
    __shared__ uint16_t wh[SORT_NW][1 << SORT_CB];
    __shared__ uint32_t tile_total;
    const int cbits = 31 - __builtin_clz((uint32_t)NBc);
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t below = (1ULL << lane) - 1;
    for (int b = threadIdx.x; b < SORT_NW * NBc; b += blockDim.x) wh[b / NBc][b % NBc] = 0;
#endif
    const int v = blockIdx.y, ch = blockIdx.x;
    for (int b = threadIdx.x; b < NBc; b += blockDim.x) {
        cur[b] = offs[cidx(v, gridDim.y, b, NBc, wmaj, ch, nch)];
        lim[b] = 0xFFFFFFFFu;
        if (slot_recs) {  // slot-relative: minus the destination's first record
            const uint32_t nbl = (uint32_t)NBc / wmaj, d = (uint32_t)b / nbl;
            const uint32_t at = d * slot_recs + hdr_recs;
            cur[b] = cur[b] - offs[cidx(0, gridDim.y, d * nbl, NBc, wmaj, 0, nch)] + at;
            lim[b] = at + cap;
        }
        lh[b] = 0;
    }
    __syncthreads();
    const uint64_t n = kr.n;
    const uint32_t fmask = (1u << fb) - 1;
    uint64_t lo = (uint64_t)ch * chunk, hi = lo + chunk < n ? lo + chunk : n;
    const uint32_t *kb = keys + ((uint64_t)v * kr.vstride + kr.off) * n;
    const bool vec = ((n | chunk) & 3) == 0;
    // the tiles of every row in one sequence, so the next tile's keys (even
    // the next row's first) are loaded while this tile goes through its LDS
    // phases: the barriers wait for LDS only, not for loads in flight
    uint32_t nxt[KPT];
    auto load_tile = [&](int r, uint64_t tb, uint32_t *key) {
        const uint32_t *k = kb + (uint64_t)r * n;
        // KPT keys per lane, in groups of four consecutive points (16-byte loads)
#pragma unroll
        for (int g = 0; g < KPT / 4; g++) {
            const uint64_t i0 = tb + 4 * (threadIdx.x + 1024 * g);
            if (vec && i0 + 4 <= hi) {
                uint4 q = *reinterpret_cast<const uint4 *>(k + i0);
                key[4 * g] = q.x; key[4 * g + 1] = q.y; key[4 * g + 2] = q.z; key[4 * g + 3] = q.w;
            } else {
#pragma unroll
                for (int j = 0; j < 4; j++) key[4 * g + j] = i0 + j < hi ? k[i0 + j] : KEY_ZERO;
            }
        }
    };
    // tile (r, tb); the next one (nr, ntb) by stepping, row by row (no 64-bit
    // division per tile)
    int r = 0;
    uint64_t tb = lo;
    if (hi > lo && kr.rows > 0) load_tile(0, lo, nxt);
    else r = kr.rows;
    while (r < kr.rows) {
        int nr = r;
        uint64_t ntb = tb + TILE_K;
        if (ntb >= hi) ntb = lo, nr++;
        const uint64_t so = v < kr.nseg ? kr.seg_off[v] : 0;
        const uint32_t idb = (uint32_t)((kr.id_row0 + r) * kr.id_mul + kr.id_base + so);
        {
            uint32_t key[KPT], rank[KPT];
#pragma unroll
            for (int j = 0; j < KPT; j++) key[j] = nxt[j];
#if PNP_SORT_PREFETCH
            if (nr < kr.rows) load_tile(nr, ntb, nxt);
#endif
#if PNP_SORT_WAVERANK
#pragma unroll
            for (int j = 0; j < KPT; j++) {
                const bool valid = key[j] != KEY_ZERO;
                const uint32_t bin = valid ? (key[j] & 0x7FFFFFFFu) >> fb : 0u;
                uint64_t peers = __ballot(valid);
                for (int b = 0; b < cbits; b++) {
                    const bool bit = (bin >> b) & 1u;
                    const uint64_t m = __ballot(bit);
                    peers &= bit ? m : ~m;
                }
                if (valid) {
                    const uint32_t base = wh[wv][bin];
                    rank[j] = base + (uint32_t)__popcll(peers & below);
                    if ((peers & below) == 0) wh[wv][bin] = (uint16_t)(base + (uint32_t)__popcll(peers));
                }
            }
            __syncthreads();
            {
                // exclusive scan of the (bin, wave) counters in bin-major order
                const int E = SORT_NW * NBc, per = (E + (int)blockDim.x - 1) / (int)blockDim.x;
                const int f0 = (int)threadIdx.x * per;
                uint32_t loc = 0;
                for (int f = f0; f < f0 + per && f < E; f++) loc += wh[f % SORT_NW][f / SORT_NW];
                const uint32_t x = wave_scan_incl(loc);
                if (lane == 63) wsum[wv] = x;
                __syncthreads();
                const uint32_t wt = wave_scan_incl(lane < SORT_NW ? wsum[lane] : 0u);
                const int wsrc = __builtin_amdgcn_readfirstlane(wv) - 1;
                uint32_t run = x - loc + (wsrc >= 0 ? (uint32_t)__builtin_amdgcn_readlane((int)wt, wsrc) : 0u);
                if (threadIdx.x == blockDim.x - 1) tile_total = run + loc;
                for (int f = f0; f < f0 + per && f < E; f++) {
                    const int b = f / SORT_NW, w = f % SORT_NW;
                    const uint32_t c = wh[w][b];
                    if (w == 0) lofs[b] = run;
                    wh[w][b] = (uint16_t)run;
                    run += c;
                }
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < KPT; j++) {
                if (key[j] == KEY_ZERO) continue;
                const uint64_t i = tb + 4 * (threadIdx.x + 1024 * (j / 4)) + (j & 3);
                uint32_t mag = key[j] & 0x7FFFFFFFu, at = wh[wv][mag >> fb] + rank[j];
                st_e[at] = (idb + (uint32_t)i) | (key[j] & 0x80000000u);
                st_m[at] = mag;
            }
            __syncthreads();
            const uint32_t total = tile_total;
            for (int b = threadIdx.x; b < NBc; b += blockDim.x)
                lh[b] = (b + 1 < NBc ? lofs[b + 1] : total) - lofs[b];
#else
#pragma unroll
            for (int j = 0; j < KPT; j++)
                if (key[j] != KEY_ZERO) rank[j] = atomicAdd(&lh[(key[j] & 0x7FFFFFFFu) >> fb], 1u);
            __syncthreads();
            tile_scan(lh, lofs, NBc, wsum);
            __syncthreads();
#pragma unroll
            for (int j = 0; j < KPT; j++) {
                if (key[j] == KEY_ZERO) continue;
                const uint64_t i = tb + 4 * (threadIdx.x + 1024 * (j / 4)) + (j & 3);
                uint32_t mag = key[j] & 0x7FFFFFFFu, at = lofs[mag >> fb] + rank[j];
                st_e[at] = (idb + (uint32_t)i) | (key[j] & 0x80000000u);
                st_m[at] = mag;
            }
            __syncthreads();
            const uint32_t total = lofs[NBc - 1] + lh[NBc - 1];
#endif
            for (uint32_t x = threadIdx.x; x < total; x += blockDim.x) {
                uint32_t mag = st_m[x], bn = mag >> fb;
                uint32_t pos = cur[bn] + x - lofs[bn];
                if (rec) {
                    if (pos < lim[bn]) rec[pos] = st_e[x] | ((uint64_t)(mag & fmask) << 32);
                } else {
                    ent[pos] = st_e[x];
                    fk[pos] = (uint16_t)(mag & fmask);
                }
            }
            __syncthreads();
            for (int b = threadIdx.x; b < NBc; b += blockDim.x) {
                cur[b] += lh[b];
                lh[b] = 0;
            }
#if PNP_SORT_WAVERANK
            for (int b = threadIdx.x; b < SORT_NW * NBc; b += blockDim.x) wh[b / NBc][b % NBc] = 0;
#endif
            __syncthreads();
        }
#if !PNP_SORT_PREFETCH
        if (nr < kr.rows) load_tile(nr, ntb, nxt);
#endif
        r = nr, tb = ntb;
    }
}

// pass B: one workgroup per (virtual window, coarse bin) = bucket range
// [p << fb, (p + 1) << fb); writes every bucket's start and the sorted entries
// Histogram first (bucket starts), then tiles of 8192 entries counting-sorted
// in LDS and written out one run per fine bin (~8 entries per fine bin and
// tile at 2^22: 8192 entries over 1024 fine bins; a coarse bin of ~106K
// entries takes ~13 tiles, the cursor h[] carrying over between them).
#ifndef PNP_TILE_F
#define PNP_TILE_F 8192
#endif
constexpr int TILE_F = PNP_TILE_F;
// PER = TILE_F / 1024 entries per lane per tile: a tile must be whole lanes,
// and st_e / st_f (6 B per entry) plus three 2^11 u32 arrays must fit in LDS
static_assert(TILE_F % 1024 == 0 && TILE_F >= 1024 && TILE_F <= 16384,
              "PNP_TILE_F must be a multiple of 1024 in [1024, 16384]");
__global__ __launch_bounds__(1024) void k_fine_sort(const uint32_t *ent, const uint16_t *fk,
                                                    const uint32_t *coffs, int nch, int fb,
                                                    uint32_t *bstart, uint32_t *sorted) {
    __shared__ uint32_t h[1 << SORT_FB_MAX], lh[1 << SORT_FB_MAX], lofs[1 << SORT_FB_MAX], wsum[16];
    __shared__ uint32_t st_e[TILE_F];
    __shared__ uint16_t st_f[TILE_F];
    const uint64_t p = blockIdx.x;
    const uint32_t ps = coffs[p * nch], pe = coffs[(p + 1) * nch];
    const int NF = 1 << fb;
    for (int f = threadIdx.x; f < NF; f += blockDim.x) h[f] = lh[f] = 0;
    __syncthreads();
    // [a, b): 4-aligned body read as 4 x u16; the rest one by one
    const uint32_t a = std::min((ps + 3) & ~3u, pe), b = std::max(pe & ~3u, a);
    {
        // four loads in flight per lane before their atomics (the loop is
        // latency-bound: ~26 steps per bin at 2^22)
        const uint32_t step = 4 * blockDim.x;
        uint32_t k = a + 4 * threadIdx.x;
        for (; k + 3 * step < b; k += 4 * step) {
            uint2 q[4];
#pragma unroll
            for (int u = 0; u < 4; u++) q[u] = *reinterpret_cast<const uint2 *>(fk + k + u * step);
#pragma unroll
            for (int u = 0; u < 4; u++) {
                atomicAdd(&h[q[u].x & 0xFFFF], 1u);
                atomicAdd(&h[q[u].x >> 16], 1u);
                atomicAdd(&h[q[u].y & 0xFFFF], 1u);
                atomicAdd(&h[q[u].y >> 16], 1u);
            }
        }
        for (; k < b; k += step) {
            const uint2 q = *reinterpret_cast<const uint2 *>(fk + k);
            atomicAdd(&h[q.x & 0xFFFF], 1u);
            atomicAdd(&h[q.x >> 16], 1u);
            atomicAdd(&h[q.y & 0xFFFF], 1u);
            atomicAdd(&h[q.y >> 16], 1u);
        }
    }
    for (uint32_t k = ps + threadIdx.x; k < a; k += blockDim.x) atomicAdd(&h[fk[k]], 1u);
    for (uint32_t k = b + threadIdx.x; k < pe; k += blockDim.x) atomicAdd(&h[fk[k]], 1u);
    __syncthreads();
    tile_scan(h, lofs, NF, wsum);
    __syncthreads();
    for (int f = threadIdx.x; f < NF; f += blockDim.x) h[f] = ps + lofs[f];  // cursor of fine bin f
    __syncthreads();
    for (int f = threadIdx.x; f < NF; f += blockDim.x) bstart[p * NF + f] = h[f];
    constexpr int PER = TILE_F / 1024;
    uint32_t ne[PER], nf[PER];
    auto load_tile = [&](uint32_t tb) {
#pragma unroll
        for (int j = 0; j < PER; j++) {
            uint32_t k = tb + threadIdx.x + j * 1024;  // coalesced, one entry per lane per step
            nf[j] = 0;
            ne[j] = 0xFFFFFFFFu;
            if (k < pe) {
                nf[j] = fk[k];
                ne[j] = ent[k];
            }
        }
    };
    if (ps < pe) load_tile(ps);
    for (uint32_t tb = ps; tb < pe; tb += TILE_F) {
        uint32_t e[PER], rank[PER];
        uint32_t f[PER];
#pragma unroll
        for (int j = 0; j < PER; j++) e[j] = ne[j], f[j] = nf[j];
#if PNP_SORT_PREFETCH
        // in flight through this tile's LDS phases (the barriers wait for LDS only)
        if (pe - tb > (uint32_t)TILE_F) load_tile(tb + TILE_F);
#endif
#pragma unroll
        for (int j = 0; j < PER; j++)
            if (tb + threadIdx.x + j * 1024 < pe) rank[j] = atomicAdd(&lh[f[j]], 1u);
        __syncthreads();
        tile_scan(lh, lofs, NF, wsum);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PER; j++) {
            uint32_t k = tb + threadIdx.x + j * 1024;
            if (k < pe) {
                uint32_t at = lofs[f[j]] + rank[j];
                st_e[at] = e[j];
                st_f[at] = f[j];
            }
        }
        __syncthreads();
        const uint32_t total = pe - tb < (uint32_t)TILE_F ? pe - tb : (uint32_t)TILE_F;
        for (uint32_t x = threadIdx.x; x < total; x += blockDim.x) {
            uint32_t bn = st_f[x];
            sorted[h[bn] + x - lofs[bn]] = st_e[x];
        }
        __syncthreads();
        for (int q = threadIdx.x; q < NF; q += blockDim.x) {
            h[q] += lh[q];
            lh[q] = 0;
        }
        __syncthreads();
#if !PNP_SORT_PREFETCH
        if (pe - tb > (uint32_t)TILE_F) load_tile(tb + TILE_F);
#endif
    }
}

// pass B over received records (bucket-range sharding): bin p's entries are
// `W` runs runs[p W + r] = {start, len} of 8-byte records (entry | fine << 32)
// in the receive buffer, one per source rank; the bin's sorted entries go to
// [out0[p], out0[p] + sum of lens) — otherwise as k_fine_sort
__global__ __launch_bounds__(1024) void k_fine_sort_runs(const uint64_t *rec, const uint2 *runs, int W,
                                                         const uint32_t *out0, int fb, uint32_t *bstart,
                                                         uint32_t *sorted) {
    __shared__ uint32_t h[1 << SORT_FB_MAX], lh[1 << SORT_FB_MAX], lofs[1 << SORT_FB_MAX], wsum[16];
    __shared__ uint32_t st_e[TILE_F];
    __shared__ uint16_t st_f[TILE_F];
    const uint64_t p = blockIdx.x;
    const int NF = 1 << fb;
    for (int f = threadIdx.x; f < NF; f += blockDim.x) h[f] = lh[f] = 0;
    __syncthreads();
    for (int r = 0; r < W; r++) {
        const uint2 run = runs[p * W + r];
        for (uint32_t k = threadIdx.x; k < run.y; k += blockDim.x)
            atomicAdd(&h[(uint32_t)(rec[run.x + k] >> 32) & 0xFFFFu], 1u);
    }
    __syncthreads();
    tile_scan(h, lofs, NF, wsum);
    __syncthreads();
    const uint32_t ps = out0[p];
    for (int f = threadIdx.x; f < NF; f += blockDim.x) h[f] = ps + lofs[f];  // cursor of fine bin f
    __syncthreads();
    for (int f = threadIdx.x; f < NF; f += blockDim.x) bstart[p * NF + f] = h[f];
    constexpr int PER = TILE_F / 1024;
    for (int r = 0; r < W; r++) {
        const uint2 run = runs[p * W + r];
        for (uint32_t tb = 0; tb < run.y; tb += TILE_F) {
            uint32_t e[PER], rank[PER], f[PER];
#pragma unroll
            for (int j = 0; j < PER; j++) {
                const uint32_t k = tb + threadIdx.x + j * 1024;
                f[j] = 0;
                if (k < run.y) {
                    const uint64_t x = rec[run.x + k];
                    e[j] = (uint32_t)x;
                    f[j] = (uint32_t)(x >> 32) & 0xFFFFu;
                    rank[j] = atomicAdd(&lh[f[j]], 1u);
                }
            }
            __syncthreads();
            tile_scan(lh, lofs, NF, wsum);
            __syncthreads();
#pragma unroll
            for (int j = 0; j < PER; j++) {
                const uint32_t k = tb + threadIdx.x + j * 1024;
                if (k < run.y) {
                    const uint32_t at = lofs[f[j]] + rank[j];
                    st_e[at] = e[j];
                    st_f[at] = (uint16_t)f[j];
                }
            }
            __syncthreads();
            const uint32_t total = run.y - tb < (uint32_t)TILE_F ? run.y - tb : (uint32_t)TILE_F;
            for (uint32_t x = threadIdx.x; x < total; x += blockDim.x) {
                const uint32_t bn = st_f[x];
                sorted[h[bn] + x - lofs[bn]] = st_e[x];
            }
            __syncthreads();
            for (int q = threadIdx.x; q < NF; q += blockDim.x) {
                h[q] += lh[q];
                lh[q] = 0;
            }
            __syncthreads();
        }
    }
}

// ---------------------------------------------------------------- 4b. fixed-slot exchange
// Slot of destination d in the send buffer (8-byte units): a header of
// hdr_recs records — u32 [0] magic, [1] this rank's record count for d, [2]
// this rank overflowed SOME slot, [3] bins per destination, [4 + p] the count
// of d's bin p (p < per_d: (MSM v, local coarse bin l) v-major) — then up to
// cap records.  Every receiver sees every sender's overflow word, so all ranks
// reach the same verdict on the batch without a host exchange.
constexpr uint32_t SLOT_MAGIC = 0x5107CA90u;
__host__ __device__ constexpr uint32_t slot_hdr_recs(uint32_t per_d) { return (4 + per_d + 1) / 2; }
__global__ __launch_bounds__(256) void k_slot_header(const uint32_t *offs, uint32_t per_d, int nch, int W,
                                                     uint32_t slot_recs, uint32_t cap, uint64_t *send,
                                                     uint32_t *dest_counts) {
    const uint32_t d = blockIdx.x;
    auto bin_off = [&](uint64_t gbin) { return offs[gbin * nch]; };
    uint32_t over = 0;
    for (int e = 0; e < W; e++) over |= bin_off((uint64_t)(e + 1) * per_d) - bin_off((uint64_t)e * per_d) > cap;
    uint32_t *h = reinterpret_cast<uint32_t *>(send + (uint64_t)d * slot_recs);
    const uint64_t g0 = (uint64_t)d * per_d;
    if (threadIdx.x == 0) {
        h[0] = SLOT_MAGIC;
        h[1] = bin_off(g0 + per_d) - bin_off(g0);
        h[2] = over;
        h[3] = per_d;
        if (dest_counts) dest_counts[d] = h[1];
    }
    for (uint32_t p = threadIdx.x; p < per_d; p += blockDim.x) h[4 + p] = bin_off(g0 + p + 1) - bin_off(g0 + p);
}

// exclusive scan over the block (1024 lanes, one value each); returns the total
__device__ uint32_t block_scan_1024(uint32_t x, uint32_t &excl, uint32_t *wsum) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t inc = x;
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(inc, off, 64);
        if (lane >= off) inc += y;
    }
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
    for (int j = 0; j < 16; j++) {
        pre += j < wv ? wsum[j] : 0;
        tot += wsum[j];
    }
    excl = pre + inc - x;
    __syncthreads();
    return tot;
}

// Receiver: from the W slot headers, the run table of k_fine_sort_runs (bin p,
// source r: {start in v_recv, length}), every bin's output start out0[p],
// the total in out0[per_d] and bstart_end, and flags = {overflow or a bad
// header, total}.  Lengths are clamped to the slot so an overflowed batch
// (redone by the caller) never reads outside it.
constexpr int SLOT_W_MAX = 64;  // ranks the fixed-slot path supports
__global__ __launch_bounds__(1024) void k_slot_runs(const uint64_t *recv, int W, uint32_t slot_recs,
                                                    uint32_t hdr_recs, uint32_t per_d, uint32_t cap, uint2 *runs,
                                                    uint32_t *out0, uint32_t *bstart_end, uint32_t *flags) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t rcarry[SLOT_W_MAX];  // records of source r in the bins already done
    __shared__ uint32_t bad;
    if (threadIdx.x == 0) bad = 0;
    if (threadIdx.x < (uint32_t)W) rcarry[threadIdx.x] = 0;
    __syncthreads();
    if (threadIdx.x < (uint32_t)W) {
        const uint32_t *h = reinterpret_cast<const uint32_t *>(recv + (uint64_t)threadIdx.x * slot_recs);
        if (h[0] != SLOT_MAGIC || h[3] != per_d || h[2]) atomicOr(&bad, 1u);
    }
    __syncthreads();
    uint32_t carry = 0;  // output records of the bins of earlier chunks
    for (uint32_t p0 = 0; p0 < per_d; p0 += 1024) {
        const uint32_t p = p0 + threadIdx.x;
        uint32_t sum = 0;
        for (int r = 0; r < W; r++) {
            const uint32_t *h = reinterpret_cast<const uint32_t *>(recv + (uint64_t)r * slot_recs);
            const uint32_t c = p < per_d ? h[4 + p] : 0;
            uint32_t pre;
            const uint32_t tot = block_scan_1024(c, pre, wsum);
            const uint32_t st = rcarry[r] + pre;  // bin p's run within source r's records
            const uint32_t len = st >= cap ? 0 : (c < cap - st ? c : cap - st);
            if (p < per_d) runs[(uint64_t)p * W + r] = make_uint2((uint32_t)r * slot_recs + hdr_recs + st, len);
            sum += len;
            __syncthreads();  // every lane has read rcarry[r]
            if (threadIdx.x == 0) rcarry[r] += tot;
        }
        uint32_t pre;
        const uint32_t tot = block_scan_1024(sum, pre, wsum);
        if (p < per_d) out0[p] = carry + pre;
        carry += tot;
    }
    if (threadIdx.x == 0) {
        out0[per_d] = carry;
        bstart_end[0] = carry;
        flags[0] = bad;
        flags[1] = carry;
    }
}

// ---------------------------------------------------------------- 5. accumulate
// balanced accumulate: thread t sums exactly the sorted entries
// [t*S, t*S + S) whatever the bucket boundaries, so every lane of a wave does
// the same number of mixed additions (one lane per bucket waits for the
// longest of 64 Poisson-sized runs: ~83% lane efficiency at n/NB = 128).  A
// bucket lying inside one thread's range is written straight to `buckets`;
// otherwise its first piece goes to tail[t0] and the pieces of the following
// threads to head[t], and msm_merge_pieces adds them up.
__device__ __forceinline__ uint32_t bucket_start(const uint32_t *offs, uint64_t u, int nch) {
    return offs[u * nch];
}
// The bucket holding sorted entry k once bucket a starts at k (start(a) == k,
// a < U): the last u >= a with start(u) <= k; `next` = start(u + 1).  Empty
// buckets (start(u + 1) == start(u)) are skipped by a galloping search — one
// load when bucket a is not empty, ~2 log2(run) for a run of empty ones.  The
// one-by-one walk it replaces made a lane crossing a whole MSM with no entries
// in a rank's bucket range (wire c over the padding rows: 65,536 empty buckets)
// issue 65,536 dependent loads: 4.7 ms on rank 7 of an 8-rank proof.
__device__ __forceinline__ uint64_t next_bucket(const uint32_t *offs, int nch, uint64_t U, uint64_t a, uint32_t k,
                                                uint32_t &next) {
    uint64_t lo = a, hi = a + 1, step = 1;
    uint32_t vhi = bucket_start(offs, hi, nch);
    while (vhi <= k) {  // start(U) = total > k: hi stays <= U
        lo = hi;
        step <<= 1;
        hi = lo + step < U ? lo + step : U;
        vhi = bucket_start(offs, hi, nch);
    }
    while (hi - lo > 1) {
        const uint64_t m = (lo + hi) >> 1;
        const uint32_t vm = bucket_start(offs, m, nch);
        if (vm <= k) lo = m;
        else hi = m, vhi = vm;
    }
    next = vhi;
    return lo;
}
// The segment walk shared by the exact kernels; `ld(e)` yields the affine
// point of sorted entry e (sign bit stripped by the caller).
// The segment walk shared by the exact kernels; `ld(e)` yields the affine
// point of sorted entry e (sign bit stripped by the caller), `st(where, i, P)`
// stores a finished piece: where = 0 bucket i, 1 head[i], 2 tail[i].
template <class LoadPt, class StorePt>
__device__ __forceinline__ void segment32(uint64_t t, LoadPt ld, StorePt st, const uint32_t *sorted,
                                          const uint32_t *offs, int nch, uint64_t U, uint32_t S) {
    const uint32_t total = bucket_start(offs, U, nch);
    const uint64_t lo64 = t * S;
    if (lo64 >= total) return;
    const uint32_t lo = (uint32_t)lo64;
    const uint32_t hi = lo + S < total ? lo + S : total;
    // largest u with start(u) <= lo: the (non-empty) bucket containing lo
    uint64_t a = 0, b = U;  // invariant: start(a) <= lo < start(b)
    while (b - a > 1) {
        uint64_t m = (a + b) >> 1;
        if (bucket_start(offs, m, nch) <= lo) a = m; else b = m;
    }
    uint64_t cur = a;
    bool first = bucket_start(offs, cur, nch) < lo;  // piece continues a bucket begun earlier
    uint32_t next = bucket_start(offs, cur + 1, nch);
    Xyzz acc = Xyzz::inf();
    for (uint32_t k = lo; k < hi; k++) {
        if (k == next) {  // bucket boundary: emit the finished piece
            if (first) st(1, t, acc);
            else st(0, cur, acc);
            first = false;
            acc = Xyzz::inf();
            cur = next_bucket(offs, nch, U, cur + 1, k, next);  // skips empty buckets
        }
        uint32_t e = sorted[k];
        Fq x, y;
        ld(e & 0x7FFFFFFFu, x, y);
        if (e >> 31) y = neg(y);
        acc = madd(acc, x, y);
    }
    if (first) st(1, t, acc);
    else if (next > hi) st(2, t, acc);
    else st(0, cur, acc);
}

__global__ __launch_bounds__(256) void k_accumulate_flat(const uint64_t *points,
                                                         const uint32_t *sorted,
                                                         const uint32_t *offs, int nch, uint64_t U,
                                                         uint32_t S, uint64_t *buckets,
                                                         uint64_t *head, uint64_t *tail) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    auto ld = [points](uint32_t i, Fq &x, Fq &y) {
        x = load_fq(points + 12ULL * i);
        y = load_fq(points + 12ULL * i + 6);
    };
    auto st = [=](int where, uint64_t i, const Xyzz &p) {
        store_xyzz((where == 0 ? buckets : where == 1 ? head : tail) + 24 * i, p);
    };
    segment32(t, ld, st, sorted, offs, nch, U, S);
}

// ---- radix-2^29 accumulation (field29.cuh) over the folded table in F29 form
// (28 u32 per point: x, y in R = 2^406 Montgomery, < 2q)
// (load29, Xyzz29: ec29.cuh)
// P += (x2, y2), madd-2008-s.  Bounds (see field29.cuh): products < 2^382,
// stored coordinates < 2^389, every product input < 2^391 (Y3 < 2^382 comes
// from mul2_29).  No equal /
// opposite / infinity cases: those make ZZ = 0 mod q, detected per piece.
// PNP_F29_KARA=1: the Karatsuba a*b halves (field29.cuh mul29k / mul2_29k, 13%
// fewer multiply-adds, same issue cycles; A/B in DESIGN.md)
#ifndef PNP_F29_KARA
#define PNP_F29_KARA 0
#endif
#if PNP_F29_KARA
#define MUL29 mul29k
#define MUL2_29 mul2_29k
#else
#define MUL29 mul29
#define MUL2_29 mul2_29
#endif
__device__ __forceinline__ void madd29(Xyzz29 &p, const F29 &x2, const F29 &y2) {
    F29 u2 = MUL29(x2, p.zz);
    F29 s2 = MUL29(y2, p.zzz);
    F29 P = sub29(u2, p.x, F29_KB);
    F29 R = sub29(s2, p.y, F29_KB);
    F29 pp = sqr29(P);
    F29 ppp = MUL29(P, pp);
    F29 q = MUL29(p.x, pp);
    F29 x3 = sub29(sub29(sub29(sqr29(R), ppp, F29_KA), q, F29_KA), q, F29_KA);
    // Y3 = R (Q - X3) - Y PPP as R (Q - X3) + Y (KA - PPP), one reduction
    F29 y3 = MUL2_29(R, sub29(q, x3, F29_KB), p.y, neg29(ppp, F29_KA));
    p.zz = MUL29(p.zz, pp);
    p.zzz = MUL29(p.zzz, ppp);
    p.x = x3;
    p.y = y3;
}
// Pieces leave the accumulation in raw radix-2^29 form (56 u32 per XYZZ
// point, 4 x 14 limbs, ec29.cuh) and stay in it through the merge and the
// reduction tree (msm_reduce.hip); only the roots are converted to R384.
// raw store; false when ZZ = 0 mod q (a degenerate step in the piece)
__device__ __forceinline__ bool store29(uint32_t *dst, const Xyzz29 &p) {
    store_f29(dst, p.x);
    store_f29(dst + 14, p.y);
    store_f29(dst + 28, p.zz);
    store_f29(dst + 42, p.zzz);
    return !zero29(p.zz);
}

#ifndef PNP_ACC_WAVES
#define PNP_ACC_WAVES 3
#endif
// Folded-table entry stride in u32: x, y (14 limbs each) padded to 128 B so a
// gathered point is exactly one cache line (112 B at a 112 B stride straddles
// two lines in 7 of 8 cases)
#ifndef PNP_PT29
#define PNP_PT29 32
#endif
static constexpr uint64_t PT29 = PNP_PT29;

// Gather staging (PNP_ACC_GLDS): the next entry's point (7 x 16 B per lane) is
// fetched global -> LDS by global_load_lds_dwordx4 while the current entry is
// added, so the ~us gather latency hides behind the addition without holding
// 28 more VGPRs (register prefetch spilled at the 3-wave budget).  Each wave
// owns 7 KiB of LDS: chunk c of lane l at stage[wave][c][l] (lane-linear, as
// the LDS-DMA destination requires).
#ifndef PNP_ACC_GLDS
#define PNP_ACC_GLDS 1
#endif
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glob_void_t;
__device__ __forceinline__ void stage_point(const uint32_t *p, uint4 *st) {
#pragma unroll
    for (int c = 0; c < 7; c++)
        __builtin_amdgcn_global_load_lds((glob_void_t *)(p + 4 * c), (lds_void_t *)(st + 64 * c), 16, 0, 0);
}
__device__ __forceinline__ void unstage_point(const uint4 *st, F29 &x, F29 &y) {
    uint32_t w[28];
#pragma unroll
    for (int c = 0; c < 7; c++) {
        const uint4 v = st[64 * c];
        w[4 * c] = v.x;
        w[4 * c + 1] = v.y;
        w[4 * c + 2] = v.z;
        w[4 * c + 3] = v.w;
    }
#pragma unroll
    for (int i = 0; i < 14; i++) {
        x.l[i] = w[i];
        y.l[i] = w[14 + i];
    }
}

__global__ __launch_bounds__(256, PNP_ACC_WAVES) void k_accumulate29(const uint32_t *pts29, const uint32_t *sorted,
                                                      const uint32_t *offs, uint64_t U, uint64_t nthr, uint32_t S,
                                                      uint32_t *buckets, uint32_t *head,
                                                      uint32_t *tail, uint32_t *tailb, uint32_t *redo,
                                                      uint32_t *nredo, uint32_t *tlist) {
#if PNP_ACC_GLDS == 1
    // per wave: the staged point (7 x 64 x 16 B) and the staged next index
    // (64 x 4 B); both arrive by LDS-DMA, so no ordinary global load result is
    // consumed inside the loop (that would make the compiler drain the DMA)
    __shared__ uint4 stage[4 * 7 * 64];
    __shared__ uint32_t sidx[4 * 64];
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    uint4 *wave_base = stage + 7 * 64 * wv;
    uint32_t *idx_base = sidx + 64 * wv;
#endif
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint32_t total = offs[U];
    S = acc_seg(offs, U, nthr, S);
    const uint64_t lo64 = t * S;
    if (lo64 >= total) return;
    const uint32_t lo = (uint32_t)lo64;
    const uint32_t hi = lo + S < total ? lo + S : total;
    uint64_t a = 0, b = U;  // start(a) <= lo < start(b)
    while (b - a > 1) {
        uint64_t m = (a + b) >> 1;
        if (offs[m] <= lo) a = m; else b = m;
    }
    uint64_t cur = a;
    bool first = offs[cur] < lo;
    uint32_t next = offs[cur + 1];
    bool ok = true, fresh = true;
    Xyzz29 acc;
#if PNP_ACC_GLDS == 1
    uint32_t e = sorted[lo];
    stage_point(pts29 + PT29 * (e & 0x7FFFFFFFu), wave_base);
    if (lo + 1 < hi)
        __builtin_amdgcn_global_load_lds((glob_void_t *)(sorted + lo + 1), (lds_void_t *)idx_base, 4, 0, 0);
#elif PNP_ACC_GLDS == 2
    // (2: the next point prefetched into registers, the index after it too)
    uint32_t e = sorted[lo];
    F29 nx = load29(pts29 + PT29 * (e & 0x7FFFFFFFu)), ny = load29(pts29 + PT29 * (e & 0x7FFFFFFFu) + 14);
    uint32_t en = lo + 1 < hi ? sorted[lo + 1] : 0u;
#endif
    for (uint32_t k = lo; k < hi; k++) {
        if (k == next) {
            ok &= store29(first ? head + 56 * t : buckets + 56 * cur, acc);
            first = false;
            fresh = true;
            cur = next_bucket(offs, 1, U, cur + 1, k, next);
        }
#if PNP_ACC_GLDS == 2
        F29 x = nx, y = ny;
        const uint32_t ecur = e;
        if (k + 1 < hi) {
            const uint32_t *p = pts29 + PT29 * (en & 0x7FFFFFFFu);
            nx = load29(p);
            ny = load29(p + 14);
            e = en;
            if (k + 2 < hi) en = sorted[k + 2];
        }
        if (ecur >> 31) y = neg29(y, F29_KA);
#elif PNP_ACC_GLDS
        F29 x, y;
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): point k and index k+1 have landed
        unstage_point(wave_base + ln, x, y);
        const uint32_t en = idx_base[ln];
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): read out before they are overwritten
        const uint32_t ecur = e;
        if (k + 1 < hi) {
            stage_point(pts29 + PT29 * (en & 0x7FFFFFFFu), wave_base);
            if (k + 2 < hi)
                __builtin_amdgcn_global_load_lds((glob_void_t *)(sorted + k + 2), (lds_void_t *)idx_base, 4, 0,
                                                 0);
            e = en;
        }
        if (ecur >> 31) y = neg29(y, F29_KA);
#else
        const uint32_t e = sorted[k];
        const uint32_t *p = pts29 + PT29 * (e & 0x7FFFFFFFu);
        F29 x = load29(p), y = load29(p + 14);
        if (e >> 31) y = neg29(y, F29_KA);
#endif
        if (fresh) {
            acc.x = x;
            acc.y = y;
            acc.zz = acc.zzz = const29(F29_ONE);
            fresh = false;
        } else {
            madd29(acc, x, y);
        }
    }
    // a bucket continuing past this segment leaves its first piece in tail[t];
    // tailb[t] names it for the merge (one merge lane per accumulation lane)
    const bool to_tail = !first && next > hi;
    ok &= store29(first ? head + 56 * t : (to_tail ? tail + 56 * t : buckets + 56 * cur), acc);
    tailb[t] = to_tail ? (uint32_t)cur : NO_TAIL;
    // the lanes with a tail, compacted (tlist[0] = count, then lane ids; one
    // atomic per wave): the merge runs one lane per listed tail instead of one
    // per accumulation lane, ~2/3 of which have none
    const uint64_t m = __ballot(to_tail);
    if (to_tail) {
        const int leader = __ffsll((unsigned long long)m) - 1;
        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        uint32_t base = 0;
        if (below == 0) base = atomicAdd(tlist, (uint32_t)__popcll(m));
        base = __shfl(base, leader);
        tlist[1 + base + below] = (uint32_t)t;
    }
    if (!ok) redo[atomicAdd(nredo, 1u)] = (uint32_t)t;
}

// Work of one k_accumulate29 launch (timed runs only, pnp_kernel_timing): the
// sorted entries E = offs[WB] and the pieces the lanes start fresh — one per
// lane with entries (ceil(E / S)) plus one per non-empty bucket whose first
// entry is not a lane's first (offs[b] % S != 0).  Every other entry is one
// mixed addition: madds = E - pieces.  ctr[0] = E, ctr[1 + (block & 63)] +=
// the block's pieces (64 counters: one atomic per 1024 buckets, spread, so
// the ~2M-bucket launch takes microseconds, not the ~0.3 ms one contended
// counter cost); the host sums them.
constexpr int WCTR_SLOTS = 64;
__global__ __launch_bounds__(1024) void k_count_pieces(const uint32_t *offs, uint64_t WB, uint64_t nthr, uint32_t S,
                                                       unsigned long long *ctr) {
    S = acc_seg(offs, WB, nthr, S);
    __shared__ uint32_t part[16];
    const uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    bool fresh = false;
    if (b < WB) {
        const uint32_t o = offs[b];
        fresh = offs[b + 1] > o && (o % S) != 0;
    }
    const unsigned long long m = __ballot(fresh);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); w++) t += part[w];
        if (t) atomicAdd(&ctr[1 + (blockIdx.x & (WCTR_SLOTS - 1))], (unsigned long long)t);
        if (blockIdx.x == 0) {
            const unsigned long long tot = offs[WB];
            ctr[0] = tot;
            atomicAdd(&ctr[1], (tot + S - 1) / S);
        }
    }
}

// exact 32-bit recomputation of the segments k_accumulate29 flagged
__global__ __launch_bounds__(64) void k_accumulate_redo(const uint32_t *pts29, const uint32_t *sorted,
                                                        const uint32_t *offs, uint64_t U, uint64_t nthr, uint32_t S,
                                                        uint32_t *buckets, uint32_t *head,
                                                        uint32_t *tail, const uint32_t *redo,
                                                        const uint32_t *nredo) {
    // grid-stride over the flagged lanes (none for random inputs: a small grid
    // that exits at once instead of one lane per accumulation lane)
    auto ld = [pts29](uint32_t i, Fq &x, Fq &y) {
        x = to_fq32(load29(pts29 + PT29 * i));
        y = to_fq32(load29(pts29 + PT29 * i + 14));
    };
    auto st = [=](int where, uint64_t i, const Xyzz &p) {
        uint32_t *d = (where == 0 ? buckets : where == 1 ? head : tail) + 56 * i;
        store_f29(d, from_fq32(p.x));
        store_f29(d + 14, from_fq32(p.y));
        store_f29(d + 28, from_fq32(p.zz));
        store_f29(d + 42, from_fq32(p.zzz));
    };
    const uint32_t cnt = *nredo;
    S = acc_seg(offs, U, nthr, S);
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < cnt; r += gridDim.x * blockDim.x)
        segment32(redo[r], ld, st, sorted, offs, 1, U, S);
}

// ---------------------------------------------------------------- folded table
// level k -> k+1: xyzz[i] = 2^c * (x, y)_i.  The c doublings run in radix
// 2^29 (ec29.cuh xdbl29, as the reduction tree's; the points of the prime-order
// group have Y != 0) between one conversion in and one out: the same canonical
// XYZZ as the 32-bit chain (PNP_TABLE_DBL29=0), 25.6 instead of 28.9 ms per
// level of 2^22 points (profiles/r04_kernel_stats_table_dbl29.csv) — part of
// the first proof after a key or SRS change.
#ifndef PNP_TABLE_DBL29
#define PNP_TABLE_DBL29 1
#endif
__global__ __launch_bounds__(256) void k_table_dbl(const uint64_t *src, uint64_t n, int c,
                                                   uint64_t *xyzz) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
#if PNP_TABLE_DBL29
    Xyzz29 q;
    q.x = from_fq32(load_fq(src + 12 * i));
    q.y = from_fq32(load_fq(src + 12 * i + 6));
    q.zz = q.zzz = const29(F29_ONE);
#pragma unroll 1
    for (int k = 0; k < c; k++) q = xdbl29(q);
    store_xyzz(xyzz + 24 * i, to32(q));
#else
    Xyzz q = dbl_affine(load_fq(src + 12 * i), load_fq(src + 12 * i + 6));
#pragma unroll 1
    for (int k = 1; k < c; k++) q = dbl(q);
    store_xyzz(xyzz + 24 * i, q);
#endif
}
// XYZZ -> affine for CH consecutive points per lane, one Fermat inversion per
// lane (Montgomery's trick over ZZZ; 1/ZZ = (ZZ/ZZZ)^2).  Points of the prime
// order group are never infinity here.
__global__ __launch_bounds__(256) void k_table_affine(const uint64_t *xyzz, uint64_t n, uint32_t CH,
                                                      uint64_t *pre, uint64_t *dst) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t lo = t * CH;
    if (lo >= n) return;
    uint64_t hi = lo + CH < n ? lo + CH : n;
    Fq acc = Fq::one();
    for (uint64_t i = lo; i < hi; i++) {
        Fq z = load_fq(xyzz + 24 * i + 18);
        if (z.is_zero()) z = Fq::one();
        acc = acc * z;
        store_fq(pre + 6 * i, acc);
    }
    Fq inv = inverse(acc);
    for (uint64_t i = hi; i-- > lo;) {
        Fq z = load_fq(xyzz + 24 * i + 18);
        const bool inf = z.is_zero();
        if (inf) z = Fq::one();
        Fq izzz = i > lo ? inv * load_fq(pre + 6 * (i - 1)) : inv;
        inv = inv * z;
        Fq w = load_fq(xyzz + 24 * i + 12) * izzz;
        Fq x = load_fq(xyzz + 24 * i) * (w * w);
        Fq y = load_fq(xyzz + 24 * i + 6) * izzz;
        if (inf) x = y = Fq::zero();
        store_fq(dst + 12 * i, x);
        store_fq(dst + 12 * i + 6, y);
    }
}

__global__ void k_table_to29(const uint64_t *T, uint64_t count, uint32_t *T29) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= count) return;
    F29 x = from_fq32(load_fq(T + 12 * i)), y = from_fq32(load_fq(T + 12 * i + 6));
    uint32_t *o = T29 + PT29 * i;
#pragma unroll
    for (int j = 0; j < 14; j++) {
        o[j] = x.l[j];
        o[14 + j] = y.l[j];
    }
}

void msm_build_table(DevBuf &tab, const uint64_t *d_points, uint64_t n, int c, hipStream_t s) {
    // level by level: each level's affine points go straight into the radix-2^29
    // table, so besides the table only two levels (n x 96 B each) live at once
    // (was: all W levels in 32-bit form first, +75% of the table's size)
    MsmCfg g = msm_cfg(n, c, true);
    const uint64_t count = (uint64_t)g.W * n;
    tab.alloc(count * PT29 * 4);
    uint32_t *T29 = static_cast<uint32_t *>(tab.p);
    const dim3 nb((uint32_t)((n + 255) / 256));
    hipLaunchKernelGGL(k_table_to29, nb, dim3(256), 0, s, d_points, n, T29);
    PNP_HIP(hipGetLastError());
    bg_step(s);
    if (g.W > 1) {
        DevBuf cur(n * 96), nxt(n * 96), xyzz(n * 192), pre(n * 48);
        const uint32_t CH = 64;
        const uint64_t lanes = (n + CH - 1) / CH;
        const uint64_t *src = d_points;
        for (int k = 1; k < g.W; k++) {
            // level k = 2^c level k-1; the top level 2^(c - top_sh) level W-2
            // (its digits are scaled by 2^top_sh, MsmCfg::top_sh)
            const int dbls = k == g.W - 1 ? g.c - g.top_sh : g.c;
            hipLaunchKernelGGL(k_table_dbl, nb, dim3(256), 0, s, src, n, dbls, xyzz.u64());
            PNP_HIP(hipGetLastError());
            bg_step(s);
            hipLaunchKernelGGL(k_table_affine, dim3((uint32_t)((lanes + 255) / 256)), dim3(256), 0, s,
                               xyzz.u64(), n, CH, pre.u64(), nxt.u64());
            PNP_HIP(hipGetLastError());
            bg_step(s);
            hipLaunchKernelGGL(k_table_to29, nb, dim3(256), 0, s, nxt.u64(), n, T29 + (uint64_t)k * n * PT29);
            PNP_HIP(hipGetLastError());
            bg_step(s);
            std::swap(cur, nxt);
            src = cur.u64();
        }
    }
    PNP_HIP(hipStreamSynchronize(s));
}

void xyzz_to_affine_dev(const uint64_t *xyzz, uint64_t n, uint64_t *aff, hipStream_t s) {
    const uint32_t CH = 64;
    const uint64_t lanes = (n + CH - 1) / CH;
    DevBuf pre(n * 48);
    hipLaunchKernelGGL(k_table_affine, dim3((uint32_t)((lanes + 255) / 256)), dim3(256), 0, s, xyzz, n, CH,
                       pre.u64(), aff);
    PNP_HIP(hipGetLastError());
    PNP_HIP(hipStreamSynchronize(s));
}

// ---------------------------------------------------------------- driver
static void put_xyzz(const Xyzz &r, uint64_t *o) {
    to_u64_limbs(r.x, o);
    to_u64_limbs(r.y, o + 6);
    to_u64_limbs(r.zz, o + 12);
    to_u64_limbs(r.zzz, o + 18);
}
static Xyzz get_xyzz(const uint64_t *e) {
    Xyzz p;
    p.x = from_u64_limbs<FqP>(e);
    p.y = from_u64_limbs<FqP>(e + 6);
    p.zz = from_u64_limbs<FqP>(e + 12);
    p.zzz = from_u64_limbs<FqP>(e + 18);
    return p;
}

// B independent MSMs over the same n points, on this GPU only; the B results
// (XYZZ) land in h_xyzz.  Per-window layout: the B*W windows are "virtual
// windows" of NB buckets each.  Folded layout (table != nullptr): virtual
// window b = MSM b with the W key rows of its windows, one bucket set.
// ---- one group of virtual windows: sort, accumulate (+ merge), reduce
struct GroupPlan {
    KeyRows kr;
    int nv;  // virtual windows (bucket sets)
};

// scalars != nullptr: the keys are not made yet; k_digits_hist makes them
// (standard folded layout: gp.kr covers every window of MSMs 0 .. nv-1)
static void sort_group(MsmWork &wk, MsmGroup &gb, const uint32_t *keys, const GroupPlan &gp,
                       const MsmCfg &g, hipStream_t s, const uint64_t *const *scalars = nullptr) {
    const int nv = gp.nv;
    const uint64_t n = gp.kr.n, WB = (uint64_t)nv * g.NB;
    // points per coarse-pass workgroup: ~512 workgroups in all, >= 1024 points each
    const int nch0 = std::max(1, 512 / std::max(nv, 1));
    const uint64_t chunk = std::max<uint64_t>(1024, (n + nch0 - 1) / nch0);
    const int nch = (int)((n + chunk - 1) / chunk);
    const int cb = std::min(SORT_CB, g.c - 1), fb = g.c - 1 - cb, NBc = 1 << cb;
    if (fb > SORT_FB_MAX) {
        set_error("msm: window of %d bits exceeds the sort's %d", g.c, SORT_CB + SORT_FB_MAX + 1);
        throw Error(PNP_E_ARG);
    }
    const uint64_t nbins = (uint64_t)nv * NBc;
    const uint64_t nent = (uint64_t)nv * gp.kr.rows * n;  // upper bound (zero digits drop out)
    auto need = [](DevBuf &b, size_t bytes) { if (b.bytes < bytes) b.alloc(bytes); };
    need(gb.counts, (nbins * nch + 1) * 4);
    need(gb.offsets, (WB + 1) * 4);
    need(gb.ent, nent * 4 + 4);
    need(gb.fkey, nent * 2 + 8);
    need(gb.sorted, nent * 4 + 4);
    uint32_t *counts = static_cast<uint32_t *>(gb.counts.p);
    uint32_t *bstart = static_cast<uint32_t *>(gb.offsets.p);
    dim3 grid((uint32_t)nch, (uint32_t)nv);
    if (scalars) {
        ScalarPtrs sp{};
        for (int v = 0; v < nv; v++) sp.p[v] = scalars[v];
        hipLaunchKernelGGL(k_digits_hist, grid, dim3(1024), 0, s, sp, n, g.c, g.W, g.top_sh, fb, NBc, chunk, nch,
                           const_cast<uint32_t *>(keys), counts, 1);
    } else {
        hipLaunchKernelGGL(k_coarse_hist, grid, dim3(1024), 0, s, keys, gp.kr, fb, NBc, chunk, nch, counts);
    }
    PNP_HIP(hipGetLastError());
    const uint64_t ncount = nbins * nch;
    PNP_HIP(hipMemsetAsync(counts + ncount, 0, 4, s));
    scan_u32(counts, ncount + 1, gb.scan_tmp, s);  // counts[ncount] = total
    uint32_t *ent = static_cast<uint32_t *>(gb.ent.p);
    uint16_t *fk = static_cast<uint16_t *>(gb.fkey.p);
    hipLaunchKernelGGL(k_coarse_scatter, grid, dim3(1024), 0, s, keys, gp.kr, fb, NBc, chunk, nch,
                       counts, ent, fk);
    PNP_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_fine_sort, dim3((uint32_t)nbins), dim3(1024), 0, s, ent, fk, counts, nch, fb,
                       bstart, static_cast<uint32_t *>(gb.sorted.p));
    PNP_HIP(hipGetLastError());
    PNP_HIP(hipMemcpyAsync(bstart + WB, counts + ncount, 4, hipMemcpyDeviceToDevice, s));
}

// entries per accumulation lane for nent sorted entries
static uint32_t acc_segment(uint64_t nent, bool folded) {
    uint32_t S = (uint32_t)std::max<uint64_t>(64, (nent >> 20) & ~7ULL);
    if (!folded) return S;
    // whole rounds of resident waves: the lane count a multiple of the chip's
    // wave slots (CUs x 4 SIMDs x PNP_ACC_WAVES x 64 lanes), so the last round
    // does not run a fraction of the chip
    static uint64_t slots = 0;
    if (!slots) {
        int dev = 0, cus = 0;
        PNP_HIP(hipGetDevice(&dev));
        PNP_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        slots = (uint64_t)cus * 4 * PNP_ACC_WAVES * 64;
    }
    const uint64_t per = (nent + slots - 1) / slots;  // entries per lane in one round
    // PNP_ACC_ROUNDS=R: at most R rounds (longer segments, fewer split buckets
    // to merge; experiments)
    static const uint64_t max_rounds = [] {
        const char *e = getenv("PNP_ACC_ROUNDS");
        return e && atoi(e) > 0 ? (uint64_t)atoi(e) : ~0ULL;
    }();
    const uint64_t rounds = std::min(max_rounds, std::max<uint64_t>(1, per / S));
    // a batch smaller than one round at S = 64 (one MSM of a 2^19-point rank
    // range: ~35 entries per lane) takes shorter segments and fills the chip
    // instead of leaving part of it idle (more bucket pieces to merge, a few %
    // of the additions)
    return (uint32_t)std::max<uint64_t>(16, (per + rounds - 1) / rounds);
}

// buckets of the group (XYZZ, R384) into gb.buckets
// nent: entries (upper bound) in the sorted list; alg_bytes: SURVEY 8(d)
// bytes credited to the launch (0: the group's points x 128 B per window)
static void accumulate_group(MsmWork &wk, MsmGroup &gb, const GroupPlan &gp, const MsmCfg &g,
                             const uint64_t *pts, const uint64_t *table, hipStream_t s, uint64_t nent = 0,
                             double alg_bytes = 0) {
    const int nv = gp.nv;
    const uint64_t n = gp.kr.n, WB = (uint64_t)nv * g.NB;
    if (!nent) nent = (uint64_t)nv * gp.kr.rows * n;
    if (alg_bytes == 0) alg_bytes = (double)n * 128.0 * nv * gp.kr.rows / g.W;
    auto need = [](DevBuf &b, size_t bytes) { if (b.bytes < bytes) b.alloc(bytes); };
    need(gb.buckets, (WB * 24 + WB * 72 + 64) * 8);  // buckets + reduction tree scratch
    const uint32_t *bstart = static_cast<const uint32_t *>(gb.offsets.p);
    const uint32_t *sorted = static_cast<const uint32_t *>(gb.sorted.p);
    uint64_t *bk = gb.buckets.u64();
    hipEvent_t ev0 = nullptr;
    if (wk.timer) wk.timer->begin("msm_accumulate", s, ev0);
    // balanced accumulate: S entries per thread, S >= 64 or ~2^20 lanes (every
    // bucket piece beyond the first costs an addition in msm_merge_pieces)
    const uint32_t S = acc_segment(nent, table != nullptr);
    const uint64_t nthr = (nent + S - 1) / S;
    if (table) {
        // raw radix-2^29 pieces: buckets inside one segment, then heads, tails
        need(gb.seg, (WB + 2 * nthr) * 224 + nthr * 4 + (nthr + 1) * 4);
        uint32_t *bk29 = static_cast<uint32_t *>(gb.seg.p);
        uint32_t *head = bk29 + 56 * WB, *tail = head + 56 * nthr, *tailb = tail + 56 * nthr;
        uint32_t *tlist = tailb + nthr;  // [0] count, then the lanes with a tail
        PNP_HIP(hipMemsetAsync(tlist, 0, 4, s));
        need(gb.redo, nthr * 4 + 16);
        uint32_t *nredo = static_cast<uint32_t *>(gb.redo.p), *redo = nredo + 4;
        PNP_HIP(hipMemsetAsync(nredo, 0, 4, s));
        const uint32_t *t29 = reinterpret_cast<const uint32_t *>(table);
        const uint32_t blocks = (uint32_t)((nthr + 255) / 256);
        hipLaunchKernelGGL(k_accumulate29, dim3(blocks), dim3(256), 0, s, t29, sorted, bstart, WB, nthr, S, bk29,
                           head, tail, tailb, redo, nredo, tlist);
        PNP_HIP(hipGetLastError());
        // equal / opposite points or infinity inside a piece: exact recomputation
        // of the flagged lanes (the count stays on the device: no host sync)
        hipLaunchKernelGGL(k_accumulate_redo, dim3((uint32_t)std::min<uint64_t>((nthr + 63) / 64, 1024)), dim3(64), 0, s, t29,
                           sorted, bstart, WB, nthr, S, bk29, head, tail, redo, nredo);
        PNP_HIP(hipGetLastError());
        // split buckets into bk29 (in place, F29; empty ones stay unwritten), reduced by msm_reduce29
        need(gb.exc, 16);
        PNP_HIP(hipMemsetAsync(gb.exc.p, 0, 4, s));
        gb.S = S;
        gb.pieces = (uint32_t)(nent / WB / S + 1);
        gb.nthr = nthr;
        need(gb.heavy, (WB + 1) * 4);
        msm_merge_pieces29(bstart, WB, S, nthr, tailb, tlist, bk29, head, tail, static_cast<uint32_t *>(gb.exc.p),
                           static_cast<uint32_t *>(gb.heavy.p), s);
    } else {
        need(gb.seg, nthr * 2 * 24 * 8);
        uint64_t *head = gb.seg.u64(), *tail = head + nthr * 24;
        hipLaunchKernelGGL(k_accumulate_flat, dim3((uint32_t)((nthr + 255) / 256)), dim3(256), 0, s, pts,
                           sorted, bstart, 1, WB, S, bk, head, tail);
        PNP_HIP(hipGetLastError());
        msm_merge_pieces(bstart, 1, WB, S, (uint32_t)(nent / WB / S + 1), head, tail, bk, s);
    }
    // algorithmic bytes: each point (96 B) and scalar (32 B)
    // once per window sweep
    if (wk.timer) {
        wk.timer->end("msm_accumulate", s, ev0, alg_bytes);
        // the dense bound nv x rows x n (zero digits drop out of the real count)
        wk.timer->credit("msm_entries_dense", (double)nent);
        if (table) {  // the real work, counted on the device (k_count_pieces)
            need(gb.wctr, 8 * (1 + WCTR_SLOTS));
            PNP_HIP(hipMemsetAsync(gb.wctr.p, 0, 8 * (1 + WCTR_SLOTS), s));
            hipLaunchKernelGGL(k_count_pieces, dim3((uint32_t)((WB + 1023) / 1024)), dim3(1024), 0, s, bstart, WB, nthr, S,
                               static_cast<unsigned long long *>(gb.wctr.p));
            PNP_HIP(hipGetLastError());
            gb.wctr_live = true;
        }
    }
}

// queue the D2H copy of a timed launch's work counters (before the caller's
// stream synchronisation) / credit them to the timer after it
static void wctr_fetch(MsmGroup &gb, hipStream_t s) {
    if (gb.wctr_live) PNP_HIP(hipMemcpyAsync(gb.wctr_h, gb.wctr.p, 8 * (1 + WCTR_SLOTS), hipMemcpyDeviceToHost, s));
}
static void wctr_credit(MsmWork &wk, MsmGroup &gb) {
    if (!gb.wctr_live) return;
    gb.wctr_live = false;
    if (!wk.timer) return;
    unsigned long long pieces = 0;
    for (int k = 1; k <= WCTR_SLOTS; k++) pieces += gb.wctr_h[k];
    wk.timer->credit("msm_entries", (double)gb.wctr_h[0]);
    wk.timer->credit("msm_madds", (double)(gb.wctr_h[0] - pieces));
}

static const uint64_t *reduce_group(MsmGroup &gb, const GroupPlan &gp, const MsmCfg &g, hipStream_t s,
                                    bool folded) {
    const uint64_t WB = (uint64_t)gp.nv * g.NB;
    uint64_t *bk = gb.buckets.u64();
    if (folded)  // radix-2^29 buckets in gb.seg, the tree in gb.buckets
        return msm_reduce29(static_cast<const uint32_t *>(gb.seg.p), static_cast<const uint32_t *>(gb.offsets.p),
                            (uint64_t)gp.nv, g.NB,
                            reinterpret_cast<uint32_t *>(bk), static_cast<uint32_t *>(gb.exc.p), s);
    return msm_reduce(bk, (uint64_t)gp.nv, g.NB, bk + WB * 24, s);
}

// the exact 32-bit merge + reduction of a folded group whose F29 pass met an
// exceptional addition (equal / opposite operands: repeated bases, crafted
// scalars); same inputs, left untouched by the F29 pass
static const uint64_t *reduce_group_exact(MsmGroup &gb, const GroupPlan &gp, const MsmCfg &g, hipStream_t s) {
    const uint64_t WB = (uint64_t)gp.nv * g.NB;
    uint64_t *bk = gb.buckets.u64();
    const uint32_t *bk29 = static_cast<const uint32_t *>(gb.seg.p);
    const uint32_t *head = bk29 + 56 * WB, *tail = head + 56 * gb.nthr;
    msm_merge_pieces29_exact(static_cast<const uint32_t *>(gb.offsets.p), WB, gb.S, gb.nthr, gb.pieces, bk29, head, tail,
                             bk, s);
    return msm_reduce(bk, (uint64_t)gp.nv, g.NB, bk + WB * 24, s);
}

static hipEvent_t ev_get(MsmWork &wk, int i) {
    if (!wk.ev[i]) PNP_HIP(hipEventCreateWithFlags(&wk.ev[i], hipEventDisableTiming));
    return wk.ev[i];
}

// B independent MSMs over the same n points, on this GPU only; the B results
// (XYZZ) land in h_xyzz.  Per-window layout: the B*W windows are "virtual
// windows" of NB buckets each.  Folded layout (table != nullptr): virtual
// window b = MSM b with the W key rows of its windows, one bucket set.
// Optionally (PNP_MSM_PIPE) the batch is split into two groups (halves of the
// MSMs, or of the windows when B = 1) pipelined over two streams: group 1's
// sort beside group 0's accumulation, group 0's bucket tree beside group 1's.
// n_table / id_base: a folded table built over n_table points of which this
// call's points are [id_base, id_base + n) (bucket-range mode keeps the full
// table; a point-range batch then indexes into it); 0 = the table is this range
static int pipe_min_b() {
    static const int v = [] {
        const char *e = getenv("PNP_MSM_PIPE");
        return e ? std::max(1, atoi(e)) : 0;
    }();
    return v;
}
static bool pipe_off() { return pipe_min_b() == 0; }

static void msm_local_batch(MsmWork &wk, const uint64_t *d_points, const uint64_t *const *d_scalars,
                            int B, uint64_t n, uint64_t *h_xyzz, hipStream_t s,
                            const uint64_t *table, uint64_t n_table = 0, uint64_t id_base = 0,
                            const uint64_t *seg_off = nullptr, int cfg_c = 0) {
    if (n == 0 || B == 0) {
        for (int b = 0; b < B; b++) put_xyzz(Xyzz::inf(), h_xyzz + 24 * b);
        return;
    }
    const bool folded = table != nullptr;
    if (!n_table) n_table = n;
    const MsmCfg g = msm_cfg(n_table, folded ? (cfg_c ? cfg_c : wk.fold_c) : 0, folded);
    auto need = [](DevBuf &b, size_t bytes) { if (b.bytes < bytes) b.alloc(bytes); };
    need(wk.digits, (uint64_t)g.W * B * n * 4);
    uint32_t *keys = static_cast<uint32_t *>(wk.digits.p);
    // PNP_MSM_FUSE_DIGITS=0: separate digit and histogram passes (A/B)
    static const bool fuse_env = [] {
        const char *e = getenv("PNP_MSM_FUSE_DIGITS");
        return !e || atoi(e) != 0;
    }();
    const bool no_pipe = pipe_off() || B < pipe_min_b();
    // the fused pass makes the keys of the single standard folded group
    const bool fuse = fuse_env && folded && B <= ScalarPtrs::MAX && no_pipe;
    if (!fuse) {
        for (int b = 0; b < B; b++) {
            hipLaunchKernelGGL(k_digits, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, d_scalars[b], n,
                               g.c, g.W, g.top_sh, keys + (uint64_t)b * g.W * n);
            PNP_HIP(hipGetLastError());
        }
    }
    // groups: (plan, first MSM of its results)
    GroupPlan gp[2];
    int ng = 1, first[2] = {0, 0};
    KeyRows kr;
    kr.n = n;
    // Two-stream pipelining measured 3% SLOWER per proof on MI355X (the sort
    // and tree kernels steal issue slots from the VALU-bound accumulation and
    // slow down themselves): one group unless PNP_MSM_PIPE=1 (experiments).
    // PNP_MSM_PIPE=B: pipeline batches of at least B MSMs only (experiments)
    if (!folded) {
        kr.vstride = 1, kr.off = 0, kr.rows = 1, kr.id_row0 = 0, kr.id_mul = 0;
        gp[0] = {kr, B * g.W};
    } else if (no_pipe) {
        kr.vstride = g.W, kr.off = 0, kr.rows = g.W, kr.id_row0 = 0, kr.id_mul = n_table;
        kr.id_base = id_base;
        gp[0] = {kr, B};
    } else if (B >= 2) {
        const int h = (B + 1) / 2;
        kr.vstride = g.W, kr.off = 0, kr.rows = g.W, kr.id_row0 = 0, kr.id_mul = n_table, kr.id_base = id_base;
        gp[0] = {kr, h};
        kr.off = h * g.W;
        gp[1] = {kr, B - h};
        first[1] = h;
        ng = 2;
    } else if (g.W >= 2) {  // one MSM: split its windows
        const int h = g.W / 2;
        kr.vstride = g.W, kr.off = 0, kr.rows = h, kr.id_row0 = 0, kr.id_mul = n_table, kr.id_base = id_base;
        gp[0] = {kr, 1};
        kr.off = h, kr.rows = g.W - h, kr.id_row0 = h;
        gp[1] = {kr, 1};
        ng = 2;
    } else {
        kr.vstride = g.W, kr.off = 0, kr.rows = g.W, kr.id_row0 = 0, kr.id_mul = n_table, kr.id_base = id_base;
        gp[0] = {kr, 1};
    }
    if (seg_off) {  // MSM first[k] + v of group k starts at seg_off[first[k] + v] (window split: MSM 0)
        for (int k = 0; k < ng; k++) {
            gp[k].kr.nseg = gp[k].nv;
            for (int v = 0; v < gp[k].nv; v++) gp[k].kr.seg_off[v] = seg_off[B == 1 ? 0 : first[k] + v];
        }
    }
    const uint64_t *pts = folded ? table : d_points;
    const uint64_t *res[2] = {nullptr, nullptr};
    if (ng == 1) {
        sort_group(wk, wk.grp[0], keys, gp[0], g, s, fuse ? d_scalars : nullptr);
        accumulate_group(wk, wk.grp[0], gp[0], g, pts, table, s);
        res[0] = reduce_group(wk.grp[0], gp[0], g, s, folded);
    } else {
        if (!wk.s2) PNP_HIP(hipStreamCreateWithFlags(&wk.s2, hipStreamNonBlocking));
        hipEvent_t evD = ev_get(wk, 0), evS1 = ev_get(wk, 1), evA0 = ev_get(wk, 2), evR0 = ev_get(wk, 3);
        PNP_HIP(hipEventRecord(evD, s));
        PNP_HIP(hipStreamWaitEvent(wk.s2, evD, 0));
        sort_group(wk, wk.grp[1], keys, gp[1], g, wk.s2);
        PNP_HIP(hipEventRecord(evS1, wk.s2));
        sort_group(wk, wk.grp[0], keys, gp[0], g, s);
        accumulate_group(wk, wk.grp[0], gp[0], g, pts, table, s);
        PNP_HIP(hipEventRecord(evA0, s));
        PNP_HIP(hipStreamWaitEvent(wk.s2, evA0, 0));
        res[0] = reduce_group(wk.grp[0], gp[0], g, wk.s2, folded);
        PNP_HIP(hipEventRecord(evR0, wk.s2));
        PNP_HIP(hipStreamWaitEvent(s, evS1, 0));
        accumulate_group(wk, wk.grp[1], gp[1], g, pts, table, s);
        res[1] = reduce_group(wk.grp[1], gp[1], g, s, folded);
        PNP_HIP(hipStreamWaitEvent(s, evR0, 0));
    }
    std::vector<uint64_t> win[2];
    uint32_t exc[2] = {0, 0}, nredo[2] = {0, 0};
    for (int k = 0; k < ng; k++) {
        win[k].resize((size_t)gp[k].nv * 24);
        PNP_HIP(hipMemcpyAsync(win[k].data(), res[k], win[k].size() * 8, hipMemcpyDeviceToHost, s));
        if (folded) {
            PNP_HIP(hipMemcpyAsync(&exc[k], wk.grp[k].exc.p, 4, hipMemcpyDeviceToHost, s));
            PNP_HIP(hipMemcpyAsync(&nredo[k], wk.grp[k].redo.p, 4, hipMemcpyDeviceToHost, s));
            wctr_fetch(wk.grp[k], s);
        }
    }
    PNP_HIP(hipStreamSynchronize(s));
    for (int k = 0; k < ng; k++) wctr_credit(wk, wk.grp[k]);
    // accumulation lanes recomputed exactly (a degenerate step in a piece)
    if (wk.timer) wk.timer->credit("msm_redo_lanes", (double)nredo[0] + nredo[1]);
    for (int k = 0; k < ng; k++) {
        if (!exc[k]) continue;
        if (wk.timer) wk.timer->credit("msm_exact_fallback", 1);
        res[k] = reduce_group_exact(wk.grp[k], gp[k], g, s);
        PNP_HIP(hipMemcpyAsync(win[k].data(), res[k], win[k].size() * 8, hipMemcpyDeviceToHost, s));
        PNP_HIP(hipStreamSynchronize(s));
    }
    if (wk.timer) wk.timer->collect();
    for (int b = 0; b < B; b++) put_xyzz(Xyzz::inf(), h_xyzz + 24 * b);
    for (int k = 0; k < ng; k++) {
        for (int v = 0; v < gp[k].nv; v++) {
            if (folded) {
                const int b = B == 1 ? 0 : first[k] + v;
                put_xyzz(add(get_xyzz(h_xyzz + 24 * b), get_xyzz(&win[k][(size_t)v * 24])), h_xyzz + 24 * b);
            }
        }
    }
    if (!folded) {
        for (int b = 0; b < B; b++) {
            Xyzz acc = Xyzz::inf();
            for (int w = g.W - 1; w >= 0; w--) {
                for (int k = 0; k < g.c; k++) acc = dbl(acc);
                acc = add(acc, get_xyzz(&win[0][((size_t)b * g.W + w) * 24]));
            }
            put_xyzz(acc, h_xyzz + 24 * b);
        }
    }
}

// One all-gather of k words per rank through the MSM exchange buffer, every
// slot closed by a tag word naming the exchange (pnp_plonk.h PNP_EX_TAG_*):
// an exchange harness can tell the messages apart without guessing from their
// sizes, and a peer whose tag differs is a rank at another point of the
// protocol (one that failed and left, or a mismatched build) — reported as
// such instead of as a garbled result.  Returns world x k words (rank-major,
// tags removed).
std::vector<uint64_t> rank_allgather(MsmWork &wk, hipStream_t s, const uint64_t *mine, int k, uint64_t tag) {
    const int W = wk.world;
    const uint64_t words = (uint64_t)k + 1, slot = 8 * words;
    if (!wk.allgather || wk.xbuf_bytes < slot * W) {
        set_error("exchange buffer %llu B < %llu B (tag %llx)", (unsigned long long)wk.xbuf_bytes,
                  (unsigned long long)(slot * W), (unsigned long long)tag);
        throw Error(PNP_E_ARG);
    }
    std::vector<uint64_t> buf(words);
    std::copy(mine, mine + k, buf.begin());
    buf[k] = tag;
    PNP_HIP(hipMemcpyAsync(wk.xbuf + words * wk.rank, buf.data(), slot, hipMemcpyHostToDevice, s));
    ex_fence(wk, s);
    if (int rc = wk.allgather(wk.user, slot)) {
        set_error("all-gather (tag %llx) failed (%d): a peer rank left the proof", (unsigned long long)tag, rc);
        throw Error(PNP_E_DEVICE);
    }
    std::vector<uint64_t> all(words * W);
    PNP_HIP(hipMemcpyAsync(all.data(), wk.xbuf, all.size() * 8, hipMemcpyDeviceToHost, s));
    PNP_HIP(hipStreamSynchronize(s));
    std::vector<uint64_t> out((size_t)k * W);
    for (int r = 0; r < W; r++) {
        if (all[words * r + k] != tag) {
            set_error("all-gather tag %llx from rank %d, expected %llx: the ranks are out of step",
                      (unsigned long long)all[words * r + k], r, (unsigned long long)tag);
            throw Error(PNP_E_DEVICE);
        }
        std::copy(all.begin() + words * r, all.begin() + words * r + k, out.begin() + (size_t)k * r);
    }
    return out;
}

// k * P on the host (double and add from k's top bit: the bucket-range weight
// offsets are < 2^19, ~20 doublings, a few microseconds each in host Fq)
static Xyzz mul_small(const Xyzz &p, uint64_t k) {
    Xyzz acc = Xyzz::inf();
    if (!k) return acc;
    for (int b = 63 - __builtin_clzll(k); b >= 0; b--) {
        acc = dbl(acc);
        if ((k >> b) & 1) acc = add(acc, p);
    }
    return acc;
}

// Bucket-range sharding of a folded batch (MsmWork::alltoallv): rank r owns
// buckets [r NB/W, (r+1) NB/W) of every MSM.  It digitises its own points
// [p0, p1) (scalars sc[b] already offset to them) and runs the usual pass A
// with 512 coarse bins, whose top log2(W) bits are the owning rank, in
// destination-major order (cidx), writing 8-byte records (entry | fine key <<
// 32) straight into the send buffer: destination d's part is one run.  After
// the all-to-all (bin counts first, then the records) every rank sorts its own
// bins from the W received runs (k_fine_sort_runs), then accumulates, merges
// and reduces only its NB/W buckets per MSM: 1/W of the bucket tail that the
// point-range scheme repeats on every rank.  Its share of MSM b is
// T_b + lo S_b (T: the local tree's weighted sum, S: the plain bucket sum,
// lo = r NB/W: the weight offset of its buckets).  Returns false (nothing
// exchanged; every rank reaches the same verdict from the all-gathered
// counts) when the records would overflow the exchange buffers: the caller
// then takes point ranges.
static bool msm_bucket_batch(MsmWork &wk, const uint64_t *const *sc, int B, uint64_t n_full, uint64_t p0,
                             uint64_t p1, uint64_t *part, hipStream_t s, const uint64_t *table,
                             const uint64_t *seg_off = nullptr, int cfg_c = 0) {
    const int W = wk.world;
    // Bucket ranges pay from 4 ranks on (solo-rank times per proof at n = 2^22,
    // points vs buckets: 2 ranks 91.1 vs 94.0 ms, 4 ranks 56.0 vs 55.3, 8 ranks
    // 37.5 vs 34.6, profiles/r03_solo): below that the extra exchange and sort
    // cost more than the halved bucket tail saves.  PNP_MSM_BUCKETS_MIN_WORLD
    // moves the threshold (tests cover 2 ranks with it).
    static const int min_world = [] {
        const char *e = getenv("PNP_MSM_BUCKETS_MIN_WORLD");
        return e ? atoi(e) : 4;
    }();
    if (W < min_world) return false;
    const MsmCfg g = msm_cfg(n_full, cfg_c ? cfg_c : wk.fold_c, true);
    int lgW = 0;
    while ((1 << lgW) < W) lgW++;
    const int cbits = std::min(SORT_CB, g.c - 1);  // coarse bits of the whole bucket index
    if ((1 << lgW) != W || lgW >= cbits || g.c - 1 - cbits > SORT_FB_MAX) return false;
    const int fb = g.c - 1 - cbits, NBc = 1 << cbits, nbl = NBc / W;  // nbl coarse bins per rank
    const uint64_t NBloc = (uint64_t)g.NB / W, n = p1 - p0;
    if (NBloc < 32) return false;
    auto need = [](DevBuf &b, size_t bytes) { if (b.bytes < bytes) b.alloc(bytes); };
    MsmGroup &gb = wk.grp[0];
    // 1. digits of this rank's points
    need(wk.digits, (uint64_t)g.W * B * std::max<uint64_t>(n, 1) * 4);
    uint32_t *keys = static_cast<uint32_t *>(wk.digits.p);
    const bool fuse = B <= ScalarPtrs::MAX;  // digits made by the histogram pass
    for (int b = 0; b < B && n && !fuse; b++) {
        hipLaunchKernelGGL(k_digits, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, sc[b], n, g.c, g.W,
                           g.top_sh, keys + (uint64_t)b * g.W * n);
        PNP_HIP(hipGetLastError());
    }
    // 2. pass A, destination-major (chunks as sort_group: ~512 workgroups)
    KeyRows kr;
    kr.n = n, kr.vstride = g.W, kr.off = 0, kr.rows = g.W, kr.id_row0 = 0, kr.id_mul = n_full, kr.id_base = p0;
    if (seg_off) {
        kr.nseg = B;
        for (int b = 0; b < B; b++) kr.seg_off[b] = seg_off[b];
    }
    const int nch0 = std::max(1, 512 / B);
    const uint64_t chunk = std::max<uint64_t>(1024, (n + nch0 - 1) / nch0);
    const int nch = (int)std::max<uint64_t>(1, (n + chunk - 1) / chunk);
    const uint64_t ncount = (uint64_t)B * NBc * nch;
    need(gb.counts, (ncount + 1) * 4);
    uint32_t *counts = static_cast<uint32_t *>(gb.counts.p);
    PNP_HIP(hipMemsetAsync(counts, 0, (ncount + 1) * 4, s));
    const dim3 grid((uint32_t)nch, (uint32_t)B);
    if (n && fuse) {
        ScalarPtrs sp{};
        for (int b = 0; b < B; b++) sp.p[b] = sc[b];
        hipLaunchKernelGGL(k_digits_hist, grid, dim3(1024), 0, s, sp, n, g.c, g.W, g.top_sh, fb, NBc, chunk, nch, keys,
                           counts, W);
        PNP_HIP(hipGetLastError());
    } else if (n) {
        hipLaunchKernelGGL(k_coarse_hist, grid, dim3(1024), 0, s, keys, kr, fb, NBc, chunk, nch, counts, W);
        PNP_HIP(hipGetLastError());
    }
    scan_u32(counts, ncount + 1, gb.scan_tmp, s);
    const uint64_t per_d = (uint64_t)B * nbl;
    const uint64_t WB = (uint64_t)B * NBloc;
    const uint64_t lo_w = (uint64_t)wk.rank * NBloc;  // weight offset of this rank's buckets
    // this batch's slot capacity (the same key, and so the same capacity, on
    // every rank: the ranks run the same batches in the same order)
    static const bool slots_on = [] {
        const char *e = getenv("PNP_MSM_SLOTS");
        return !(e && atoi(e) == 0);
    }();
    if (wk.slot_cap.size() > 1024) wk.slot_cap.clear();  // (operator-API batches never repeat a key)
    const auto key = std::make_tuple(wk.batch_seq++, B, n_full);
    const uint32_t hdr = slot_hdr_recs((uint32_t)per_d);
    auto cap_it = wk.slot_cap.find(key);
    if (slots_on && W <= SLOT_W_MAX && cap_it != wk.slot_cap.end()) {
        // ---- fixed slots: no host round trip before the accumulation
        // (PNP_TEST_SLOT_CAP: a smaller capacity, to exercise the overflow path)
        static const uint64_t test_cap = [] {
            const char *e = getenv("PNP_TEST_SLOT_CAP");
            return e ? strtoull(e, nullptr, 0) : 0ULL;
        }();
        const uint64_t cap = test_cap ? std::min(test_cap, cap_it->second) : cap_it->second;
        const uint64_t slot_recs = hdr + cap;
        // u32 layout of slot_dev: runs (2 per_d W) | out0 (per_d + 1) | flags (2) | dest counts (W)
        const uint64_t nruns = 2 * per_d * W;
        need(wk.slot_dev, (nruns + per_d + 1 + 2 + W) * 4);
        uint32_t *rt = static_cast<uint32_t *>(wk.slot_dev.p), *o0 = rt + nruns, *flags = o0 + per_d + 1,
                 *dcnt = flags + 2;
        hipLaunchKernelGGL(k_slot_header, dim3((uint32_t)W), dim3(256), 0, s, counts, (uint32_t)per_d, nch, W,
                           (uint32_t)slot_recs, (uint32_t)cap, wk.v_send, dcnt);
        PNP_HIP(hipGetLastError());
        if (n) {
            hipLaunchKernelGGL(k_coarse_scatter, grid, dim3(1024), 0, s, keys, kr, fb, NBc, chunk, nch, counts,
                               nullptr, nullptr, W, wk.v_send, (uint32_t)slot_recs, hdr, (uint32_t)cap);
            PNP_HIP(hipGetLastError());
        }
        ex_fence(wk, s);
        std::vector<uint64_t> eq(W, slot_recs * 8);
        if (int rc = wk.alltoallv(wk.v_user, eq.data(), eq.data())) {
            set_error("msm bucket shard: slot all-to-all failed (%d)", rc);
            throw Error(PNP_E_DEVICE);
        }
        need(gb.offsets, (WB + 1) * 4);
        need(gb.sorted, W * cap * 4 + 4);
        uint32_t *bstart = static_cast<uint32_t *>(gb.offsets.p);
        hipLaunchKernelGGL(k_slot_runs, dim3(1), dim3(1024), 0, s, wk.v_recv, W, (uint32_t)slot_recs, hdr,
                           (uint32_t)per_d, (uint32_t)cap, reinterpret_cast<uint2 *>(rt), o0, bstart + WB, flags);
        PNP_HIP(hipGetLastError());
        hipLaunchKernelGGL(k_fine_sort_runs, dim3((uint32_t)per_d), dim3(1024), 0, s, wk.v_recv,
                           reinterpret_cast<const uint2 *>(rt), W, o0, fb, bstart,
                           static_cast<uint32_t *>(gb.sorted.p));
        PNP_HIP(hipGetLastError());
        MsmCfg gl = g;
        gl.NB = (int)NBloc;
        GroupPlan gp;
        gp.kr = kr;
        gp.nv = B;
        // (the record count stays on the device: W cap bounds the lanes, the
        // kernels read the true total from bstart[WB])
        accumulate_group(wk, gb, gp, gl, nullptr, table, s, W * cap, (double)W * cap * 128.0 / g.W);
        const uint64_t *res = reduce_group(gb, gp, gl, s, true);
        std::vector<uint64_t> ts((size_t)B * 48);
        uint32_t exc = 0, nredo = 0, fl[2] = {0, 0};
        std::vector<uint32_t> dc(W);
        PNP_HIP(hipMemcpyAsync(ts.data(), res, ts.size() * 8, hipMemcpyDeviceToHost, s));
        PNP_HIP(hipMemcpyAsync(&exc, gb.exc.p, 4, hipMemcpyDeviceToHost, s));
        PNP_HIP(hipMemcpyAsync(&nredo, gb.redo.p, 4, hipMemcpyDeviceToHost, s));
        PNP_HIP(hipMemcpyAsync(fl, flags, 8, hipMemcpyDeviceToHost, s));
        PNP_HIP(hipMemcpyAsync(dc.data(), dcnt, 4 * W, hipMemcpyDeviceToHost, s));
        wctr_fetch(gb, s);
        PNP_HIP(hipStreamSynchronize(s));
        wk.slot_runs++;
        if (fl[0]) {
            // some rank overflowed some slot (every rank saw its flag): the
            // variable path below redoes the batch and raises the capacity
            gb.wctr_live = false;
            wk.slot_overflows++;
            if (wk.timer) {
                wk.timer->credit("msm_slot_overflows", 1);
                wk.timer->collect();
            }
        } else {
            wctr_credit(wk, gb);
            if (wk.timer) {
                wk.timer->credit("msm_slot_batches", 1);
                wk.timer->credit("msm_redo_lanes", (double)nredo);
                uint64_t mx = 0, sum = 0;
                for (uint32_t c : dc) mx = std::max<uint64_t>(mx, c), sum += c;
                wk.timer->credit("msm_dest_max", (double)mx);
                wk.timer->credit("msm_dest_sum", (double)sum);
            }
            if (exc) {
                if (wk.timer) wk.timer->credit("msm_exact_fallback", 1);
                res = reduce_group_exact(gb, gp, gl, s);
                PNP_HIP(hipMemcpyAsync(ts.data(), res, ts.size() * 8, hipMemcpyDeviceToHost, s));
                PNP_HIP(hipStreamSynchronize(s));
            }
            if (wk.timer) wk.timer->collect();
            for (int b = 0; b < B; b++) {
                const Xyzz T = get_xyzz(&ts[24 * (size_t)b]), S = get_xyzz(&ts[24 * ((size_t)B + b)]);
                put_xyzz(lo_w ? add(T, mul_small(S, lo_w)) : T, part + 24 * (size_t)b);
            }
            return true;
        }
    }
    // ---- variable sizes: the counts travel first (host round trips)
    std::vector<uint32_t> offs(ncount + 1);
    PNP_HIP(hipMemcpyAsync(offs.data(), counts, (ncount + 1) * 4, hipMemcpyDeviceToHost, s));
    PNP_HIP(hipStreamSynchronize(s));
    // per destination: its bins' entry counts (B nbl words, bin (v, local) of
    // destination d starts at offs[((d B + v) nbl + l) nch]) and its record bytes
    auto bin_off = [&](uint64_t gbin) { return offs[gbin * nch]; };
    std::vector<uint64_t> send_b(W), recv_b(W);
    for (int d = 0; d < W; d++) send_b[d] = 8ULL * (bin_off((d + 1) * per_d) - bin_off(d * per_d));
    // 3. every rank's totals (one all-gather of W words per rank): the
    // receive sizes and the common overflow verdict
    const std::vector<uint64_t> all = rank_allgather(wk, s, send_b.data(), W, PNP_EX_TAG_COUNTS);
    auto cnt = [&](int from, int to) { return all[(size_t)from * W + to]; };
    const uint64_t bins_bytes = 4 * per_d * W;  // the bin-count exchange below
    bool fits = bins_bytes <= wk.v_bytes;
    for (int r = 0; r < W; r++) {
        uint64_t out = 0, in = 0;
        for (int d = 0; d < W; d++) {
            out += cnt(r, d);
            in += cnt(d, r);
        }
        fits &= out <= wk.v_bytes && in <= wk.v_bytes;
    }
    if (!fits) {
        if (wk.timer) wk.timer->credit("msm_bucket_fallback", 1);
        return false;
    }
    {
        // the slot capacity of this batch for the next proofs: the largest
        // (source, destination) count of this run + 3% + 256 records (the
        // balance over proofs of one circuit is within ~1%)
        uint64_t mx = 0;
        for (uint64_t v : all) mx = std::max<uint64_t>(mx, v / 8);
        const uint64_t cap = ((mx + mx / 32 + 256) + 63) & ~63ULL;
        if (W <= SLOT_W_MAX && (uint64_t)W * (hdr + cap) * 8 <= wk.v_bytes && cap < (1ULL << 31)) {
            uint64_t &c = wk.slot_cap[key];
            c = std::max(c, cap);
        }
        if (wk.timer) {
            uint64_t smx = 0, sum = 0;
            for (int d = 0; d < W; d++) smx = std::max<uint64_t>(smx, send_b[d] / 8), sum += send_b[d] / 8;
            wk.timer->credit("msm_dest_max", (double)smx);
            wk.timer->credit("msm_dest_sum", (double)sum);
        }
    }
    for (int r = 0; r < W; r++) recv_b[r] = cnt(r, wk.rank);
    // 4. bin counts (u32, B nbl per destination), then the records.  `bc`
    // lives until the stream synchronisation below: in ordered mode nothing
    // waits for its upload before then
    std::vector<uint32_t> bc((size_t)per_d * W);
    {
        for (uint64_t gbin = 0; gbin < per_d * W; gbin++) bc[gbin] = bin_off(gbin + 1) - bin_off(gbin);
        PNP_HIP(hipMemcpyAsync(wk.v_send, bc.data(), bc.size() * 4, hipMemcpyHostToDevice, s));
        ex_fence(wk, s);
        std::vector<uint64_t> eq(W, 4 * per_d);
        if (int rc = wk.alltoallv(wk.v_user, eq.data(), eq.data())) {
            set_error("msm bucket shard: bin-count all-to-all failed (%d)", rc);
            throw Error(PNP_E_DEVICE);
        }
    }
    std::vector<uint32_t> rbc((size_t)per_d * W);  // [source][v][local bin]
    PNP_HIP(hipMemcpyAsync(rbc.data(), wk.v_recv, rbc.size() * 4, hipMemcpyDeviceToHost, s));
    if (n) {
        hipLaunchKernelGGL(k_coarse_scatter, grid, dim3(1024), 0, s, keys, kr, fb, NBc, chunk, nch, counts,
                           nullptr, nullptr, W, wk.v_send);
        PNP_HIP(hipGetLastError());
    }
    PNP_HIP(hipStreamSynchronize(s));
    if (int rc = wk.alltoallv(wk.v_user, send_b.data(), recv_b.data())) {
        set_error("msm bucket shard: all-to-all failed (%d)", rc);
        throw Error(PNP_E_DEVICE);
    }
    // 5. the W received runs of every bin (v, local coarse bin) and its output start
    std::vector<uint32_t> runs(2 * per_d * W), out0(per_d + 1);
    {
        uint64_t base = 0;
        for (int r = 0; r < W; r++) {
            uint64_t at = base;
            for (uint64_t p = 0; p < per_d; p++) {
                const uint32_t c = rbc[(size_t)r * per_d + p];
                runs[2 * (p * W + r)] = (uint32_t)at;
                runs[2 * (p * W + r) + 1] = c;
                at += c;
            }
            if (at - base != recv_b[r] / 8) {
                set_error("msm bucket shard: rank %d sent %llu records, its bin counts say %llu", r,
                          (unsigned long long)(recv_b[r] / 8), (unsigned long long)(at - base));
                throw Error(PNP_E_DEVICE);
            }
            base = at;
        }
        uint64_t o = 0;
        for (uint64_t p = 0; p < per_d; p++) {
            out0[p] = (uint32_t)o;
            for (int r = 0; r < W; r++) o += runs[2 * (p * W + r) + 1];
        }
        out0[per_d] = (uint32_t)o;
    }
    const uint64_t R = out0[per_d];
    need(gb.offsets, (WB + 1) * 4);
    need(gb.sorted, R * 4 + 4);
    need(gb.ent, (runs.size() + out0.size()) * 4);  // run table + bin starts (ent is unused on this path)
    uint32_t *bstart = static_cast<uint32_t *>(gb.offsets.p);
    uint32_t *rt = static_cast<uint32_t *>(gb.ent.p), *o0 = rt + runs.size();
    PNP_HIP(hipMemcpyAsync(rt, runs.data(), runs.size() * 4, hipMemcpyHostToDevice, s));
    PNP_HIP(hipMemcpyAsync(o0, out0.data(), out0.size() * 4, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_fine_sort_runs, dim3((uint32_t)per_d), dim3(1024), 0, s, wk.v_recv,
                       reinterpret_cast<const uint2 *>(rt), W, o0, fb, bstart, static_cast<uint32_t *>(gb.sorted.p));
    PNP_HIP(hipGetLastError());
    PNP_HIP(hipMemcpyAsync(bstart + WB, o0 + per_d, 4, hipMemcpyDeviceToDevice, s));
    // 6. accumulate, merge and reduce this rank's buckets
    MsmCfg gl = g;
    gl.NB = (int)NBloc;
    GroupPlan gp;
    gp.kr = kr;
    gp.nv = B;
    std::vector<uint64_t> ts((size_t)B * 48);
    for (int b = 0; b < 2 * B; b++) put_xyzz(Xyzz::inf(), &ts[24 * (size_t)b]);
    if (R) {
        accumulate_group(wk, gb, gp, gl, nullptr, table, s, R, (double)R * 128.0 / g.W);
        const uint64_t *res = reduce_group(gb, gp, gl, s, true);
        uint32_t exc = 0, nredo = 0;
        PNP_HIP(hipMemcpyAsync(ts.data(), res, ts.size() * 8, hipMemcpyDeviceToHost, s));
        PNP_HIP(hipMemcpyAsync(&exc, gb.exc.p, 4, hipMemcpyDeviceToHost, s));
        PNP_HIP(hipMemcpyAsync(&nredo, gb.redo.p, 4, hipMemcpyDeviceToHost, s));
        wctr_fetch(gb, s);
        PNP_HIP(hipStreamSynchronize(s));
        wctr_credit(wk, gb);
        if (wk.timer) wk.timer->credit("msm_redo_lanes", (double)nredo);
        if (exc) {
            if (wk.timer) wk.timer->credit("msm_exact_fallback", 1);
            res = reduce_group_exact(gb, gp, gl, s);
            PNP_HIP(hipMemcpyAsync(ts.data(), res, ts.size() * 8, hipMemcpyDeviceToHost, s));
            PNP_HIP(hipStreamSynchronize(s));
        }
        if (wk.timer) wk.timer->collect();
    }
    for (int b = 0; b < B; b++) {
        const Xyzz T = get_xyzz(&ts[24 * (size_t)b]), S = get_xyzz(&ts[24 * ((size_t)B + b)]);
        put_xyzz(lo_w ? add(T, mul_small(S, lo_w)) : T, part + 24 * (size_t)b);
    }
    return true;
}

int msm_fold_c(uint64_t n_points, int fold_c) { return msm_cfg(n_points, fold_c, true).c; }

// ---- HBM of the MSM machinery (upper bounds for the key-load budget,
// abi.cpp hbm_plan; checked against the measured peak by tests/test_gpu_hbm.py)
uint64_t msm_table_bytes(uint64_t n_points, uint64_t n_cfg, int fold_c) {
    return (uint64_t)msm_cfg(n_cfg, fold_c, true).W * n_points * PT29 * 4;
}
uint64_t msm_table_build_bytes(uint64_t n_points) { return n_points * (96 + 96 + 192 + 48); }
// a batch of B folded MSMs over n_pts points of a table configured for n_cfg;
// world > 1 with v_bytes > 0: bucket ranges (1/world of the buckets, at most
// v_bytes / 8 received records accumulated), else point ranges / one GPU
uint64_t msm_work_bytes(uint64_t n_pts, uint64_t n_cfg, int fold_c, int B, uint64_t v_bytes, int world) {
    const MsmCfg g = msm_cfg(n_cfg, fold_c, true);
    const bool buckets = world > 1 && v_bytes > 0;
    const uint64_t WB = (uint64_t)B * (buckets ? g.NB / world : g.NB);
    const uint64_t nent = (uint64_t)B * g.W * n_pts;  // the dense bound the buffers are sized for
    const uint64_t digits = nent * 4, counts = (uint64_t)B * 512 * 1024 * 4 + (WB + 1) * 4;
    // point ranges: pass-A entries + fine keys + sorted entries; bucket
    // ranges: the received records sorted into `sorted`
    const uint64_t acc_ent = buckets ? v_bytes / 8 : nent;
    const uint64_t sort = buckets ? acc_ent * 4 : nent * (4 + 2 + 4);
    const uint64_t S = std::max<uint32_t>(16, acc_segment(acc_ent, true));
    const uint64_t nthr = (acc_ent + S - 1) / S;
    const uint64_t acc = (WB + 2 * nthr) * 224 + nthr * 12 + (WB + 1) * 4 + (WB * 24 + WB * 72 + 64) * 8;
    return digits + counts + sort + acc;
}
uint64_t msm_work_held(const MsmWork &wk) {
    uint64_t b = wk.digits.bytes + wk.part_counts.bytes + wk.rec_counts.bytes;
    for (const MsmGroup &g : wk.grp)
        b += g.counts.bytes + g.offsets.bytes + g.scan_tmp.bytes + g.ent.bytes + g.fkey.bytes + g.sorted.bytes +
             g.buckets.bytes + g.seg.bytes + g.redo.bytes + g.exc.bytes + g.heavy.bytes + g.wctr.bytes;
    return b;
}

void msm_point_range(uint64_t n, int rank, int world, uint64_t &p0, uint64_t &p1) {
    const uint64_t per = (n + world - 1) / world;
    p0 = std::min<uint64_t>((uint64_t)rank * per, n);
    p1 = std::min<uint64_t>(p0 + per, n);
}

// Multi-GPU: rank r takes the points [p0, p1) of msm_point_range (every
// window; the folded table passed in covers that range), the B partial sums
// meet in one all-gather of B XYZZ points per rank and are added on the host.
void msm_run_batch(MsmWork &wk, const uint64_t *d_points, const uint64_t *const *d_scalars, int B,
                   uint64_t n, uint64_t *h_xyzz, hipStream_t s, const uint64_t *table,
                   bool scalars_local, const MsmSegs *segs) {
    if (segs && (!table || B > MSM_BATCH_MAX)) {
        set_error("msm: point segments need a folded table and at most %d MSMs", MSM_BATCH_MAX);
        throw Error(PNP_E_ARG);
    }
    if (wk.timer) wk.timer->credit("msm_scalar_bytes", 32.0 * (double)B * n / wk.world);  // (this rank's scalars)
    if (wk.world == 1) {
        if (segs)
            msm_local_batch(wk, nullptr, d_scalars, B, n, h_xyzz, s, table, segs->n_table, 0, segs->off, segs->c);
        else
            msm_local_batch(wk, d_points, d_scalars, B, n, h_xyzz, s, table);
        return;
    }
    uint64_t p0, p1;
    msm_point_range(n, wk.rank, wk.world, p0, p1);
    std::vector<const uint64_t *> sc(B);
    for (int b = 0; b < B; b++) sc[b] = scalars_local ? d_scalars[b] : d_scalars[b] + 4 * p0;
    std::vector<uint64_t> part((size_t)B * 24);
    // bucket ranges (the folded table covers all n points) or point ranges; a
    // segmented table covers every point of its sets, or (sliced) this rank's
    // range of each
    const bool full = table && (wk.full_table() || (segs && !segs->sliced));
    const uint64_t n_tab = segs ? segs->n_table : n;
    const uint64_t *off = segs ? segs->off : nullptr;
    if (segs && segs->sliced && wk.full_table()) {
        set_error("msm: a sliced segment table in bucket-range mode");
        throw Error(PNP_E_ARG);
    }
    const int cc = segs ? segs->c : 0;
    if (!(table && wk.full_table() &&
          msm_bucket_batch(wk, sc.data(), B, n_tab, p0, p1, part.data(), s, table, off, cc)))
        msm_local_batch(wk, d_points ? d_points + 12 * p0 : nullptr, sc.data(), B, p1 - p0, part.data(), s, table,
                        segs ? n_tab : full ? n_tab : 0, full ? p0 : 0, off, cc);
    const std::vector<uint64_t> all = rank_allgather(wk, s, part.data(), B * 24, PNP_EX_TAG_MSM_SUMS);
    for (int b = 0; b < B; b++) {
        Xyzz acc = Xyzz::inf();
        for (int r = 0; r < wk.world; r++) acc = add(acc, get_xyzz(&all[((size_t)r * B + b) * 24]));
        put_xyzz(acc, h_xyzz + 24 * b);
    }
}

void msm_run(MsmWork &wk, const uint64_t *d_points, const uint64_t *d_scalars, uint64_t n,
             uint64_t *h_xyzz, hipStream_t s, const uint64_t *table) {
    const uint64_t *sc[1] = {d_scalars};
    msm_run_batch(wk, d_points, sc, 1, n, h_xyzz, s, table);
}

void xyzz_to_affine_host(const uint64_t *xyzz, uint64_t *aff12) { xyzz_to_affine_batch_host(xyzz, 1, aff12); }

// B results at once with ONE Fq inversion (Montgomery's trick over ZZ ZZZ;
// 1/ZZ = ZZZ / (ZZ ZZZ), 1/ZZZ = ZZ / (ZZ ZZZ)): the host converts every
// batch of commitments between two GPU phases, and a Fermat inversion costs
// tens of microseconds on the CPU
void xyzz_to_affine_batch_host(const uint64_t *xyzz, int B, uint64_t *aff12) {
    std::vector<Xyzz> p(B);
    std::vector<Fq> pre(B + 1);
    pre[0] = Fq::one();
    for (int b = 0; b < B; b++) {
        p[b] = get_xyzz(xyzz + 24 * b);
        pre[b + 1] = p[b].is_inf() ? pre[b] : pre[b] * (p[b].zz * p[b].zzz);
    }
    Fq inv = inverse(pre[B]);  // 1 / prod(ZZ ZZZ) over the finite points
    for (int b = B - 1; b >= 0; b--) {
        uint64_t *o = aff12 + 12 * b;
        if (p[b].is_inf()) {  // (0, one) as the reference's to_affine (point.cu:29-36)
            to_u64_limbs(Fq::zero(), o);
            to_u64_limbs(Fq::one(), o + 6);
            continue;
        }
        const Fq d = inv * pre[b];  // 1 / (ZZ ZZZ)
        inv = inv * (p[b].zz * p[b].zzz);
        to_u64_limbs(p[b].x * (p[b].zzz * d), o);
        to_u64_limbs(p[b].y * (p[b].zz * d), o + 6);
    }
}

}  // namespace pnp
