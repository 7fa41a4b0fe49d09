// msm.hip — Pippenger MSM on BLS12-381 G1 for gfx950.
//
// Contract of the reference's multi_scalar_mult (utils/function.cu:275-290 ->
// zksnark_msm.cu:45-83 -> sppark_msm/pippenger.cuh:470-556, CPU fold in
// zkp/cpu/collect.h:326-489): sum_i s_i * P_i for n affine Montgomery points
// and n scalars (here Montgomery in, canonicalised on the device, as
// to_base in PLONK/src/arithmetic.cu:3-8).
//
// MI355X design (no cooperative kernels, no CPU bucket fold):
//   1. k_digits     : signed c-bit digits, |d| <= 2^(c-1), one u16 key per
//                     (window, point) — key = (|d|-1) | sign<<15, 0xFFFF = 0.
//   2. k_hist       : one workgroup per (window, chunk of points) builds the
//                     chunk's bucket histogram in LDS (2^(c-1) u32 <= 128 KiB)
//                     and stores it bucket-major, chunk-minor.
//   3. scan         : exclusive scan of those counts = the start of every
//                     (window, bucket, chunk) run in the sorted index list.
//   4. k_scatter    : same workgroups place point indices with LDS cursors —
//                     no global atomics anywhere.
//   5. k_accumulate : one lane per (window, bucket) walks its run and sums the
//                     points in XYZZ with mixed additions (8M + 2S).
//   6. k_reduce     : window sums sum_b b*B_b by a running-sum tree:
//                     groups of 8 entries merge as T' = sum T + len * sum t*S.
//   7. host         : Horner over the windows (c doublings each) + affine.
#include <algorithm>
#include "pnp_internal.h"
#include "ec.cuh"

namespace pnp {

struct MsmCfg {
    int c, W, NB, nch;
    uint64_t chunk;
};

static MsmCfg msm_cfg(uint64_t n) {
    MsmCfg g;
    int lg = 0;
    while ((1ULL << lg) < n) lg++;
    g.c = lg >= 20 ? 16 : (lg - 3 < 4 ? 4 : lg - 3);
    g.W = (256 + g.c - 1) / g.c;
    g.NB = 1 << (g.c - 1);
    g.chunk = n < 8192 ? 8192 : (n >> 4 < 8192 ? 8192 : n >> 4);  // <= 16 chunks per window
    g.nch = (int)((n + g.chunk - 1) / g.chunk);
    return g;
}

// ---------------------------------------------------------------- 1. digits
__global__ void k_digits(const uint64_t *scalars, uint64_t n, int c, int W, uint16_t *keys) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fr s = from_mont(load_fr(scalars, i));
    const uint32_t NB = 1u << (c - 1);
    uint32_t carry = 0;
    for (int w = 0; w < W; w++) {
        int bit = w * c;
        int li = bit >> 5, sh = bit & 31;
        uint64_t word = li < 8 ? s.v[li] : 0;
        if (li + 1 < 8) word |= (uint64_t)s.v[li + 1] << 32;
        uint32_t raw = (uint32_t)(word >> sh) & ((1u << c) - 1);
        raw += carry;
        uint16_t key = 0xFFFF;
        if (raw > NB) {
            uint32_t mag = (NB << 1) - raw;  // |raw - 2^c|, 0 when raw = 2^c
            carry = 1;
            if (mag) key = (uint16_t)((mag - 1) | 0x8000u);
        } else {
            carry = 0;
            if (raw) key = (uint16_t)(raw - 1);
        }
        // for c = 16 the top window never carries (scalars < 2^255)
        keys[(uint64_t)w * n + i] = key;
    }
}

// ---------------------------------------------------------------- 2. histogram
__global__ __launch_bounds__(1024) void k_hist(const uint16_t *keys, uint64_t n, int NB,
                                               uint64_t chunk, int nch, uint32_t *counts) {
    extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
    const int w = blockIdx.y, ch = blockIdx.x;
    for (int b = threadIdx.x; b < NB; b += blockDim.x) hist[b] = 0;
    __syncthreads();
    uint64_t lo = (uint64_t)ch * chunk, hi = lo + chunk < n ? lo + chunk : n;
    const uint16_t *k = keys + (uint64_t)w * n;
    for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        uint16_t key = k[i];
        if (key != 0xFFFF) atomicAdd(&hist[key & 0x7FFF], 1u);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < NB; b += blockDim.x)
        counts[((uint64_t)w * NB + b) * nch + ch] = hist[b];
}

// ---------------------------------------------------------------- 3. scan
// exclusive scan of u32 in place, three phases over 1024-element tiles
__global__ __launch_bounds__(256) void k_scan_tiles(uint32_t *d, uint64_t n, uint32_t *tile_sums) {
    __shared__ uint32_t s[1024];
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
    (void)s;
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

// ---------------------------------------------------------------- 4. scatter
__global__ __launch_bounds__(1024) void k_scatter(const uint16_t *keys, uint64_t n, int NB,
                                                  uint64_t chunk, int nch, const uint32_t *offs,
                                                  uint32_t *sorted) {
    extern __shared__ __attribute__((aligned(16))) uint32_t cur[];
    const int w = blockIdx.y, ch = blockIdx.x;
    for (int b = threadIdx.x; b < NB; b += blockDim.x) cur[b] = offs[((uint64_t)w * NB + b) * nch + ch];
    __syncthreads();
    uint64_t lo = (uint64_t)ch * chunk, hi = lo + chunk < n ? lo + chunk : n;
    const uint16_t *k = keys + (uint64_t)w * n;
    for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        uint16_t key = k[i];
        if (key == 0xFFFF) continue;
        uint32_t pos = atomicAdd(&cur[key & 0x7FFF], 1u);
        sorted[pos] = (uint32_t)i | ((uint32_t)(key >> 15) << 31);
    }
}

// ---------------------------------------------------------------- 5. accumulate
__global__ __launch_bounds__(256) void k_accumulate(const uint64_t *points, const uint32_t *sorted,
                                                    const uint32_t *offs, int NB, int nch, int W,
                                                    uint64_t *buckets) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (t >= (uint64_t)W * NB) return;
    uint32_t start = offs[t * nch];
    uint32_t end = offs[(t + 1) * nch];  // offs[W*NB*nch] = total (sentinel)
    Xyzz acc = Xyzz::inf();
    for (uint32_t k = start; k < end; k++) {
        uint32_t e = sorted[k];
        uint32_t idx = e & 0x7FFFFFFFu;
        const uint64_t *p = points + 12ULL * idx;
        Fq x = load_fq(p), y = load_fq(p + 6);
        if (e >> 31) y = neg(y);
        acc = madd(acc, x, y);
    }
    store_xyzz(buckets + 24 * t, acc);
}

// 5'. balanced accumulate: thread t sums exactly the sorted entries
// [t*S, t*S + S) whatever the bucket boundaries, so every lane of a wave does
// the same number of mixed additions (one lane per bucket waits for the
// longest of 64 Poisson-sized runs: ~83% lane efficiency at n/NB = 128).  A
// bucket lying inside one thread's range is written straight to `buckets`;
// otherwise its first piece goes to tail[t0] and the pieces of the following
// threads to head[t], and k_bucket_merge adds them up.
__device__ __forceinline__ uint32_t bucket_start(const uint32_t *offs, uint64_t u, int nch) {
    return offs[u * nch];
}
__global__ __launch_bounds__(256) void k_accumulate_flat(const uint64_t *points,
                                                         const uint32_t *sorted,
                                                         const uint32_t *offs, int nch, uint64_t U,
                                                         uint32_t S, uint64_t *buckets,
                                                         uint64_t *head, uint64_t *tail) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
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
            if (first) store_xyzz(head + 24 * t, acc);
            else store_xyzz(buckets + 24 * cur, acc);
            first = false;
            acc = Xyzz::inf();
            do {  // skip empty buckets
                cur++;
                next = bucket_start(offs, cur + 1, nch);
            } while (next == k);
        }
        uint32_t e = sorted[k];
        const uint64_t *p = points + 12ULL * (e & 0x7FFFFFFFu);
        Fq x = load_fq(p), y = load_fq(p + 6);
        if (e >> 31) y = neg(y);
        acc = madd(acc, x, y);
    }
    if (first) store_xyzz(head + 24 * t, acc);
    else if (next > hi) store_xyzz(tail + 24 * t, acc);
    else store_xyzz(buckets + 24 * cur, acc);
}

// bucket u = tail[t0] + head[t0+1] + ... + head[t1] when its entries span
// threads t0 < t1; empty buckets become infinity
__global__ __launch_bounds__(256) void k_bucket_merge(const uint32_t *offs, int nch, uint64_t U,
                                                      uint32_t S, const uint64_t *head,
                                                      const uint64_t *tail, uint64_t *buckets) {
    uint64_t u = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (u >= U) return;
    uint32_t s = bucket_start(offs, u, nch), e = bucket_start(offs, u + 1, nch);
    if (s == e) {
        store_xyzz(buckets + 24 * u, Xyzz::inf());
        return;
    }
    uint32_t t0 = s / S, t1 = (e - 1) / S;
    if (t0 == t1) return;
    Xyzz acc = load_xyzz(tail + 24ULL * t0);
    for (uint32_t t = t0 + 1; t <= t1; t++) acc = add(acc, load_xyzz(head + 24ULL * t));
    store_xyzz(buckets + 24 * u, acc);
}

// ---------------------------------------------------------------- 6. reduce
// Entry e of a level stands for a contiguous bucket range of length `len`
// (power of two): T_e = sum_r (r+1) B_r over the range, S_e = sum_r B_r.
// Groups of G entries merge into one: T' = sum_t T_t + len * sum_t t * S_t.
// Leaves: T = S = B.
template <int G>
__global__ __launch_bounds__(256) void k_reduce(const uint64_t *inT, const uint64_t *inS,
                                                uint64_t nout, uint32_t lg_len, uint64_t *outT,
                                                uint64_t *outS) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (t >= nout) return;
    Xyzz sumT = Xyzz::inf(), run = Xyzz::inf(), acc = Xyzz::inf();
#pragma unroll 1
    for (int k = G - 1; k >= 0; k--) {
        uint64_t e = t * G + k;
        Xyzz T = load_xyzz(inT + 24 * e);
        Xyzz S = load_xyzz(inS + 24 * e);
        sumT = add(sumT, T);
        if (k > 0) {
            run = add(run, S);
            acc = add(acc, run);  // after the loop: acc = sum_{t>=1} t * S_t
        } else {
            run = add(run, S);
        }
    }
    for (uint32_t d = 0; d < lg_len; d++) acc = dbl(acc);
    store_xyzz(outT + 24 * t, add(sumT, acc));
    store_xyzz(outS + 24 * t, run);
}

// B independent MSMs over the same n points: the B*W windows are treated as
// one set of "virtual windows" so every stage runs once for the whole batch.
void msm_run_batch(MsmWork &wk, const uint64_t *d_points, const uint64_t *const *d_scalars, int B,
                   uint64_t n, uint64_t *h_xyzz, hipStream_t s) {
    if (n == 0 || B == 0) {
        Xyzz r = Xyzz::inf();
        for (int b = 0; b < B; b++) {
            uint64_t *o = h_xyzz + 24 * b;
            to_u64_limbs(r.x, o); to_u64_limbs(r.y, o + 6); to_u64_limbs(r.zz, o + 12);
            to_u64_limbs(r.zzz, o + 18);
        }
        return;
    }
    MsmCfg g = msm_cfg(n);
    const int WW = g.W * B;  // virtual windows (c-bit windows x batched MSMs)
    // window sharding: rank r owns virtual windows [v0, v0 + nown)
    const int per = (WW + wk.world - 1) / wk.world;
    const int v0 = std::min(wk.rank * per, WW);
    const int nown = std::min(v0 + per, WW) - v0;
    const uint64_t WB = (uint64_t)nown * g.NB;
    auto need = [](DevBuf &b, size_t bytes) { if (b.bytes < bytes) b.alloc(bytes); };
    need(wk.digits, (uint64_t)WW * n * 2);
    need(wk.counts, (WB * g.nch + 1) * 4);
    need(wk.sorted, (uint64_t)nown * n * 4);
    need(wk.buckets, (WB + WB / 2 + 64 * (uint64_t)nown) * 24 * 8);
    uint16_t *keys = static_cast<uint16_t *>(wk.digits.p);
    uint32_t *counts = static_cast<uint32_t *>(wk.counts.p);
    uint32_t *sorted = static_cast<uint32_t *>(wk.sorted.p);

    const uint64_t *inT = nullptr;
    if (nown > 0) {
        for (int b = 0; b < B; b++) {
            if ((b + 1) * g.W <= v0 || b * g.W >= v0 + nown) continue;  // no owned window
            hipLaunchKernelGGL(k_digits, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s,
                               d_scalars[b], n, g.c, g.W, keys + (uint64_t)b * g.W * n);
            PNP_HIP(hipGetLastError());
        }
        const uint16_t *own_keys = keys + (uint64_t)v0 * n;
        dim3 grid((uint32_t)g.nch, (uint32_t)nown);
        size_t lds = (size_t)g.NB * 4;
        static bool attr_set = false;
        if (!attr_set) {
            PNP_HIP(hipFuncSetAttribute((const void *)k_hist,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
            PNP_HIP(hipFuncSetAttribute((const void *)k_scatter,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
            attr_set = true;
        }
        hipLaunchKernelGGL(k_hist, grid, dim3(1024), lds, s, own_keys, n, g.NB, g.chunk, g.nch,
                           counts);
        PNP_HIP(hipGetLastError());
        const uint64_t ncount = WB * g.nch;
        PNP_HIP(hipMemsetAsync(counts + ncount, 0, 4, s));
        scan_u32(counts, ncount + 1, wk.offsets, s);  // counts[ncount] = total
        hipLaunchKernelGGL(k_scatter, grid, dim3(1024), lds, s, own_keys, n, g.NB, g.chunk, g.nch,
                           counts, sorted);
        PNP_HIP(hipGetLastError());
        uint64_t *bk = wk.buckets.u64();
        hipEvent_t ev0 = nullptr;
        if (wk.timer) wk.timer->begin("msm_accumulate", s, ev0);
        // balanced accumulate: S entries per thread (upper bound nown*n entries)
        const uint32_t S = 64;
        const uint64_t nthr = ((uint64_t)nown * n + S - 1) / S;
        need(wk.seg, nthr * 2 * 24 * 8);
        uint64_t *head = wk.seg.u64(), *tail = head + nthr * 24;
        hipLaunchKernelGGL(k_accumulate_flat, dim3((uint32_t)((nthr + 255) / 256)), dim3(256), 0,
                           s, d_points, sorted, counts, g.nch, WB, S, bk, head, tail);
        PNP_HIP(hipGetLastError());
        hipLaunchKernelGGL(k_bucket_merge, dim3((uint32_t)((WB + 255) / 256)), dim3(256), 0, s,
                           counts, g.nch, WB, S, head, tail, bk);
        PNP_HIP(hipGetLastError());
        // algorithmic bytes: each point (96 B) and scalar (32 B)
        // once per owned window-sweep
        if (wk.timer)
            wk.timer->end("msm_accumulate", s, ev0, (double)n * 128.0 * nown / g.W);
        // running-sum tree: per virtual window NB entries -> 1
        const uint64_t *inS = bk;
        inT = bk;
        uint64_t *free_ptr = bk + WB * 24;
        uint64_t m = WB;
        uint32_t lg_len = 0;
        uint64_t per_win = g.NB;
        while (per_win > 1) {
            int G = per_win >= 8 ? 8 : (int)per_win;
            uint64_t nout = m / G;
            uint64_t *oT = free_ptr, *oS = free_ptr + nout * 24;
            free_ptr += 2 * nout * 24;
            uint32_t blocks = (uint32_t)((nout + 255) / 256);
            switch (G) {
                case 8: hipLaunchKernelGGL(k_reduce<8>, dim3(blocks), dim3(256), 0, s, inT, inS, nout, lg_len, oT, oS); break;
                case 4: hipLaunchKernelGGL(k_reduce<4>, dim3(blocks), dim3(256), 0, s, inT, inS, nout, lg_len, oT, oS); break;
                case 2: hipLaunchKernelGGL(k_reduce<2>, dim3(blocks), dim3(256), 0, s, inT, inS, nout, lg_len, oT, oS); break;
                default: set_error("msm reduce"); throw Error(PNP_E_ARG);
            }
            PNP_HIP(hipGetLastError());
            inT = oT;
            inS = oS;
            m = nout;
            per_win /= G;
            lg_len += (G == 8 ? 3 : G == 4 ? 2 : 1);
        }
    }
    std::vector<uint64_t> win((size_t)WW * 24);
    if (wk.world == 1) {
        PNP_HIP(hipMemcpyAsync(win.data(), inT, win.size() * 8, hipMemcpyDeviceToHost, s));
        PNP_HIP(hipStreamSynchronize(s));
    } else {
        // slot r of xbuf = windows [r*per, r*per + per): the gathered buffer is
        // window-indexed, so one copy brings all WW window sums to the host
        const uint64_t slot = (uint64_t)per * 24 * 8;
        if (wk.xbuf_bytes < slot * wk.world) {
            set_error("msm shard: exchange buffer %llu B < %llu B",
                      (unsigned long long)wk.xbuf_bytes, (unsigned long long)(slot * wk.world));
            throw Error(PNP_E_ARG);
        }
        if (nown > 0)
            PNP_HIP(hipMemcpyAsync(wk.xbuf + (uint64_t)v0 * 24, inT, (uint64_t)nown * 24 * 8,
                                   hipMemcpyDeviceToDevice, s));
        PNP_HIP(hipStreamSynchronize(s));
        int rc = wk.allgather(wk.user, slot);
        if (rc != 0) {
            set_error("msm shard: all-gather callback failed (%d)", rc);
            throw Error(PNP_E_DEVICE);
        }
        PNP_HIP(hipMemcpyAsync(win.data(), wk.xbuf, win.size() * 8, hipMemcpyDeviceToHost, s));
        PNP_HIP(hipStreamSynchronize(s));
    }
    if (wk.timer) wk.timer->collect();
    for (int b = 0; b < B; b++) {
        Xyzz acc = Xyzz::inf();
        for (int w = g.W - 1; w >= 0; w--) {
            for (int k = 0; k < g.c; k++) acc = dbl(acc);
            const uint64_t *e = &win[((size_t)b * g.W + w) * 24];
            Xyzz ww;
            ww.x = from_u64_limbs<FqP>(e);
            ww.y = from_u64_limbs<FqP>(e + 6);
            ww.zz = from_u64_limbs<FqP>(e + 12);
            ww.zzz = from_u64_limbs<FqP>(e + 18);
            acc = add(acc, ww);
        }
        uint64_t *o = h_xyzz + 24 * b;
        to_u64_limbs(acc.x, o);
        to_u64_limbs(acc.y, o + 6);
        to_u64_limbs(acc.zz, o + 12);
        to_u64_limbs(acc.zzz, o + 18);
    }
}

void msm_run(MsmWork &wk, const uint64_t *d_points, const uint64_t *d_scalars, uint64_t n,
             uint64_t *h_xyzz, hipStream_t s) {
    const uint64_t *sc[1] = {d_scalars};
    msm_run_batch(wk, d_points, sc, 1, n, h_xyzz, s);
}

void xyzz_to_affine_host(const uint64_t *xyzz, uint64_t *aff12) {
    Xyzz p;
    p.x = from_u64_limbs<FqP>(xyzz);
    p.y = from_u64_limbs<FqP>(xyzz + 6);
    p.zz = from_u64_limbs<FqP>(xyzz + 12);
    p.zzz = from_u64_limbs<FqP>(xyzz + 18);
    Fq x, y;
    xyzz_to_affine(p, x, y);
    to_u64_limbs(x, aff12);
    to_u64_limbs(y, aff12 + 6);
}

}  // namespace pnp
