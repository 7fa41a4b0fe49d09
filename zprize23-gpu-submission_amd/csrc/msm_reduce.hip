// msm_reduce.hip — Pippenger bucket reduction: sum_b (b+1) B_b per window.
//
// Replaces the reference's per-window running sum on the GPU plus the CPU
// fold (sppark_msm/pippenger.cuh:360-468, zkp/cpu/collect.h:326-489).
//
// The reduction has little work (a few additions per bucket) and is bound by
// the LATENCY of dependent XYZZ additions (~22 us each on one lane, measured
// with tools/ubench_chain.hip), so it is organised for depth, not work:
// a binary tree over the buckets of each window where a node of height h
// covering buckets [a, a + 2^h) carries
//     S = sum B_b,   T = sum (b - a + 1) B_b,   D = 2^h S.
// Children L, R (height h-1) combine as
//     S = S_L + S_R,   T = (T_L + T_R) + D_R,   D = 2 (D_L + D_R),
// four additions and one doubling of depth 2 per level, so a window of 2^15
// buckets is reduced at depth ~30 instead of the ~150 of running sums whose
// partial results are scaled by repeated doubling.  The root's T is the window
// sum.  One launch per level, one lane per node.
#include "msm_internal.h"
#include "ec.cuh"
#include "ec29.cuh"

namespace pnp {

// leaves (h = 1) from bucket pairs: S = B0 + B1, T = S + B1, D = 2 S
__global__ __launch_bounds__(256) void k_tree_leaf(const uint64_t *bk, uint64_t nout, uint64_t *out) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (t >= nout) return;
    Xyzz b1 = load_xyzz(bk + 24 * (2 * t + 1));
    Xyzz S = add(load_xyzz(bk + 24 * (2 * t)), b1);
    uint64_t *o = out + 72 * t;
    store_xyzz(o, S);
    store_xyzz(o + 24, add(S, b1));
    store_xyzz(o + 48, dbl(S));
}

// leaves of height log2(LW) from LW buckets by running sums (right to left):
// S = sum B_k, T = sum (k+1) B_k, D = LW S.  Throughput-friendlier than the
// pairwise leaf when the window has many buckets (2 additions per bucket,
// depth ~LW additions + log2(LW) doublings).
#ifndef PNP_LEAF_W
#define PNP_LEAF_W 8
#endif
template <int LW>
__global__ __launch_bounds__(256) void k_tree_leafw(const uint64_t *bk, uint64_t nout, uint64_t *out) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (t >= nout) return;
    const uint64_t *b = bk + 24 * LW * t;
    Xyzz S = load_xyzz(b + 24 * (LW - 1)), T = S;
#pragma unroll 1
    for (int k = LW - 2; k >= 0; k--) {
        S = add(S, load_xyzz(b + 24 * k));
        T = add(T, S);
    }
    uint64_t *o = out + 72 * t;
    store_xyzz(o, S);
    store_xyzz(o + 24, T);
    Xyzz D = S;
#pragma unroll 1
    for (int k = 1; k < LW; k *= 2) D = dbl(D);
    store_xyzz(o + 48, D);
}

// node t from nodes 2t, 2t+1 of the level below; triples (S, T, D) of 72 u64.
// Three lanes per node, one per component (blockIdx.y, so every wave runs one
// path: divergent components would serialise 1 + 2 + 2 operations), each at
// most two operations deep.
__global__ __launch_bounds__(256) void k_tree_level(const uint64_t *in, uint64_t nout, uint64_t *out) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (t >= nout) return;
    const int c = (int)blockIdx.y;
    const uint64_t *L = in + 144 * t, *R = L + 72;
    Xyzz r;
    if (c == 0) {
        r = add(load_xyzz(L), load_xyzz(R));
    } else if (c == 1) {
        r = add(add(load_xyzz(L + 24), load_xyzz(R + 24)), load_xyzz(R + 48));
    } else {
        r = dbl(add(load_xyzz(L + 48), load_xyzz(R + 48)));
    }
    store_xyzz(out + 72 * t + 24 * c, r);
}

// G lanes per bucket (G | 256, a power of two): lane j sums pieces j, j+G,
// ... serially, then a log2(G)-step LDS tree.  G is chosen so that every lane
// adds ~4 pieces: the merge is latency-bound (~22 us per dependent addition).
__global__ __launch_bounds__(256) void k_merge_pieces(const uint32_t *offs, int nch, uint64_t U,
                                                      uint32_t S, int G, const uint64_t *head,
                                                      const uint64_t *tail, uint64_t *bk) {
    __shared__ uint64_t lds[256 * 24];
    const uint64_t g = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / G;
    const int j = threadIdx.x % G;
    bool live = false;
    Xyzz acc = Xyzz::inf();
    if (g < U) {
        uint32_t s0 = offs[g * nch], e0 = offs[(g + 1) * nch];
        if (s0 == e0) {
            if (j == 0) store_xyzz(bk + 24 * g, Xyzz::inf());
        } else {
            uint32_t t0 = s0 / S, t1 = (e0 - 1) / S;
            if (t0 != t1) {
                live = true;
                // piece k = tail[t0] (k = 0) or head[t0 + k]
#pragma unroll 1
                for (uint32_t k = j; k <= t1 - t0; k += G)
                    acc = add(acc, load_xyzz(k == 0 ? tail + 24ULL * t0 : head + 24ULL * (t0 + k)));
            }
        }
    }
    uint64_t *mine = lds + 24 * threadIdx.x;
    for (int h = G / 2; h >= 1; h /= 2) {
        store_xyzz(mine, acc);
        __syncthreads();
        if (live && j < h) acc = add(acc, load_xyzz(mine + 24 * h));
        __syncthreads();
    }
    if (live && j == 0) store_xyzz(bk + 24 * g, acc);
}

void msm_merge_pieces(const uint32_t *offs, int nch, uint64_t U, uint32_t S, uint32_t pieces,
                      const uint64_t *head, const uint64_t *tail, uint64_t *bk, hipStream_t s) {
    int G = 1;
    while (G < 8 && (uint32_t)G * 8 <= pieces) G *= 2;
    const uint64_t blocks = (U * G + 255) / 256;
    hipLaunchKernelGGL(k_merge_pieces, dim3((uint32_t)blocks), dim3(256), 0, s, offs, nch, U, S, G,
                       head, tail, bk);
    PNP_HIP(hipGetLastError());
}

// Folded layout: the pieces are raw radix-2^29 XYZZ points (56 u32, msm.hip
// store29) and stay in radix 2^29 (ec29.cuh: shorter dependent chains than
// the 32-bit Fq products, no per-piece conversion).  A bucket inside one
// lane's segment is already bk29[u].  A bucket u split across lanes t0 < t1 is
// tail29[t0] + head29[t0+1] + ... + head29[t1]; its merge lane is accumulation
// lane t0, which recorded u in tailb[t0] and listed itself in tlist.  Empty buckets are not written
// (msm_reduce29 reads them as infinity).  A bucket of more than MERGE_HEAVY
// pieces (clustered or repeated scalars, a short top window) is not summed
// here, where one lane would add its pieces one after another, but queued
// for k_merge_heavy29.
// (16, not 64: a bucket of 16-63 pieces was one lane's chain of dependent
// additions — at 8 ranks the wires' repeated values made round 1's merge a
// 0.85 ms chain; same box, solo rank 0 of 8: 30.2 -> 29.5 ms per proof, one
// GPU neutral, profiles/r05_ab_merge_heavy.txt)
#ifndef PNP_MERGE_HEAVY
#define PNP_MERGE_HEAVY 16
#endif
constexpr uint32_t MERGE_HEAVY = PNP_MERGE_HEAVY;
// One merge lane per listed tail (tlist: the accumulation lanes that left
// one, compacted by k_accumulate29): a wave is 64 merges, where one lane per
// accumulation lane ran ~1 in 3 of its lanes (a segment of ~3 buckets splits one)
__global__ __launch_bounds__(256) void k_merge_tails29(const uint32_t *offs, uint64_t U, uint64_t nthr, uint32_t S,
                                                       const uint32_t *tailb, const uint32_t *tlist, uint32_t *bk29,
                                                       const uint32_t *head, const uint32_t *tail, uint32_t *exc,
                                                       uint32_t *heavy, uint32_t *nheavy) {
    const uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (q >= tlist[0]) return;
    S = acc_seg(offs, U, nthr, S);
    const uint64_t t = tlist[1 + q];
    const uint32_t u = tailb[t];
    const uint32_t t1 = (offs[u + 1] - 1) / S;
    if (t1 - (uint32_t)t >= MERGE_HEAVY) {
        heavy[atomicAdd(nheavy, 1u)] = u;
        return;
    }
    Xyzz29 acc = load_xyzz29(tail + 56 * t);
#pragma unroll 1
    for (uint32_t k = (uint32_t)t + 1; k <= t1; k++) acc = xadd29_inf(acc, load_xyzz29(head + 56ULL * k), exc);
    store_xyzz29(bk29 + 56ULL * u, acc);
}

// the queued heavy buckets, one workgroup each (grid-stride over the queue):
// 256 lanes sum every 256th piece, then an LDS tree of log2 of the lanes that
// hold a piece (8 levels from 128 pieces on, 4 for a bucket of 16)
__global__ __launch_bounds__(256) void k_merge_heavy29(const uint32_t *offs, uint64_t U, uint64_t nthr, uint32_t S,
                                                       uint32_t *bk29, const uint32_t *head, const uint32_t *tail,
                                                       uint32_t *exc, const uint32_t *heavy, const uint32_t *nheavy) {
    __shared__ uint32_t lds[256 * 56];
    const uint32_t cnt = *nheavy;
    S = acc_seg(offs, U, nthr, S);
    uint32_t *mine = lds + 56 * threadIdx.x;
    for (uint32_t q = blockIdx.x; q < cnt; q += gridDim.x) {
        const uint32_t g = heavy[q];
        const uint32_t t0 = offs[g] / S, t1 = (offs[g + 1] - 1) / S;
        Xyzz29 acc = inf29();
#pragma unroll 1
        for (uint32_t k = threadIdx.x; k <= t1 - t0; k += blockDim.x)
            acc = xadd29_inf(acc, load_xyzz29(k == 0 ? tail + 56ULL * t0 : head + 56ULL * (t0 + k)), exc);
        // lanes >= the piece count hold infinity: the tree starts at the
        // power of two that covers the pieces
        uint32_t h0 = 1;
        while (2 * h0 < t1 - t0 + 1 && 2 * h0 < blockDim.x) h0 *= 2;
        for (uint32_t h = h0; h >= 1; h /= 2) {
            store_xyzz29(mine, acc);
            __syncthreads();
            if (threadIdx.x < h) acc = xadd29_inf(acc, load_xyzz29(mine + 56 * h), exc);
            __syncthreads();
        }
        if (threadIdx.x == 0) store_xyzz29(bk29 + 56ULL * g, acc);
        __syncthreads();
    }
}

void msm_merge_pieces29(const uint32_t *offs, uint64_t U, uint32_t S, uint64_t nthr, const uint32_t *tailb,
                        const uint32_t *tlist, uint32_t *bk29, const uint32_t *head, const uint32_t *tail,
                        uint32_t *exc, uint32_t *heavy, hipStream_t s) {
    uint32_t *nheavy = heavy, *list = heavy + 1;
    PNP_HIP(hipMemsetAsync(nheavy, 0, 4, s));
    // (the count stays on the device: a grid for every accumulation lane, the
    // waves past the count exit at once)
    hipLaunchKernelGGL(k_merge_tails29, dim3((uint32_t)((nthr + 255) / 256)), dim3(256), 0, s, offs, U, nthr, S,
                       tailb, tlist, bk29, head, tail, exc, list, nheavy);
    PNP_HIP(hipGetLastError());
    // a small grid: it exits at once when nothing was queued
    hipLaunchKernelGGL(k_merge_heavy29, dim3(256), dim3(256), 0, s, offs, U, nthr, S, bk29, head, tail, exc, list,
                       nheavy);
    PNP_HIP(hipGetLastError());
}

// The exact fallback of the F29 merge + tree (an exceptional addition was
// flagged): every piece converted to R384 and summed with ec.cuh's add; a
// bucket inside one lane's segment is bk29[u] as the accumulation left it
// (the F29 merge writes only split and empty buckets).  Writes bk (R384) for
// the 32-bit msm_reduce.
__device__ __forceinline__ Xyzz piece29(const uint32_t *p) { return to32(load_xyzz29(p)); }
__global__ __launch_bounds__(256) void k_merge_pieces29_exact(const uint32_t *offs, uint64_t U, uint64_t nthr,
                                                              uint32_t S, int G, const uint32_t *bk29,
                                                              const uint32_t *head, const uint32_t *tail,
                                                              uint64_t *bk) {
    __shared__ uint64_t lds[256 * 24];
    S = acc_seg(offs, U, nthr, S);
    const uint64_t g = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / G;
    const int j = threadIdx.x % G;
    bool live = false;
    Xyzz acc = Xyzz::inf();
    if (g < U) {
        uint32_t s0 = offs[g], e0 = offs[g + 1];
        if (s0 != e0) {
            live = true;
            uint32_t t0 = s0 / S, t1 = (e0 - 1) / S;
            if (t0 == t1) {
                if (j == 0) acc = piece29(bk29 + 56 * g);
            } else {
#pragma unroll 1
                for (uint32_t k = j; k <= t1 - t0; k += G)
                    acc = add(acc, piece29(k == 0 ? tail + 56ULL * t0 : head + 56ULL * (t0 + k)));
            }
        } else if (j == 0) {
            store_xyzz(bk + 24 * g, Xyzz::inf());
        }
    }
    uint64_t *mine = lds + 24 * threadIdx.x;
    for (int h = G / 2; h >= 1; h /= 2) {
        store_xyzz(mine, acc);
        __syncthreads();
        if (live && j < h) acc = add(acc, load_xyzz(mine + 24 * h));
        __syncthreads();
    }
    if (live && j == 0) store_xyzz(bk + 24 * g, acc);
}

void msm_merge_pieces29_exact(const uint32_t *offs, uint64_t U, uint32_t S, uint64_t nthr, uint32_t pieces,
                              const uint32_t *bk29, const uint32_t *head, const uint32_t *tail, uint64_t *bk,
                              hipStream_t s) {
    int G = 1;
    while (G < 8 && (uint32_t)G * 8 <= pieces) G *= 2;
    const uint64_t blocks = (U * G + 255) / 256;
    hipLaunchKernelGGL(k_merge_pieces29_exact, dim3((uint32_t)blocks), dim3(256), 0, s, offs, U, nthr, S, G, bk29,
                       head, tail, bk);
    PNP_HIP(hipGetLastError());
}

// radix-2^29 tree: the (S, T, D) nodes of k_tree_leafw / k_tree_level, 168
// u32 per node
// (bucket u empty, offs[u] = offs[u + 1]: infinity, bk29[u] unwritten)
__device__ __forceinline__ Xyzz29 bucket29(const uint32_t *bk, const uint32_t *offs, uint64_t u) {
    return offs[u] == offs[u + 1] ? inf29() : load_xyzz29(bk + 56 * u);
}
// Running sums from the top bucket down: S = sum_(j>=k) B_j, T = sum (j-k+1) B_j.
// T == S as points exactly while the only non-empty bucket above k is k + 1
// (T - S = sum_(j>k+1) (j-k-1) B_j): then an EMPTY bucket k makes the update
// T + S a doubling, which the incomplete addition cannot do (it would flag the
// whole group for the exact 32-bit redo).  `tis` tracks T == S; that step is
// done as 2 T.  Empty buckets are rare at 2^22 points (~100 entries per
// bucket) but not at the 2^19-point ranks of an 8-GPU proof (~13: e^-13 per
// bucket, ~2 such leaves per proof).
template <int LW>
__global__ __launch_bounds__(256) void k_tree_leafw29(const uint32_t *bk, const uint32_t *offs, uint64_t nout,
                                                      uint32_t *out, uint32_t *exc) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (t >= nout) return;
    const uint64_t u0 = (uint64_t)LW * t;
    Xyzz29 S = bucket29(bk, offs, u0 + LW - 1), T = S;
    bool tis = true;  // T == S
#pragma unroll 1
    for (int k = LW - 2; k >= 0; k--) {
        const bool empty = offs[u0 + k] == offs[u0 + k + 1];
        if (empty) {
            // S unchanged; T + S = 2 T when T == S
            T = tis ? xdbl29_inf(T) : xadd29_inf(T, S, exc);
            tis = tis && zero29(T.zz);  // still equal only while both are infinity
        } else {
            S = xadd29_inf(S, load_xyzz29(bk + 56 * (u0 + k)), exc);
            const bool tinf = zero29(T.zz);
            T = xadd29_inf(T, S, exc);  // T != S here: S gained a bucket T lacks
            tis = tinf;                 // inf + S = S
        }
    }
    uint32_t *o = out + 168 * t;
    store_xyzz29(o, S);
    store_xyzz29(o + 56, T);
    Xyzz29 D = S;
#pragma unroll 1
    for (int k = 1; k < LW; k *= 2) D = xdbl29_inf(D);
    store_xyzz29(o + 112, D);
}

__global__ __launch_bounds__(256) void k_tree_level29(const uint32_t *in, uint64_t nout, uint32_t *out,
                                                      uint32_t *exc) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (t >= nout) return;
    const int c = (int)blockIdx.y;
    const uint32_t *L = in + 336 * t, *R = L + 168;
    Xyzz29 r;
    if (c == 0) {
        r = xadd29_inf(load_xyzz29(L), load_xyzz29(R), exc);
    } else if (c == 1) {
        r = xadd29_inf(xadd29_inf(load_xyzz29(L + 56), load_xyzz29(R + 56), exc), load_xyzz29(R + 112), exc);
    } else {
        r = xdbl29_inf(xadd29_inf(load_xyzz29(L + 112), load_xyzz29(R + 112), exc));
    }
    store_xyzz29(out + 168 * t + 56 * c, r);
}

// ---- the tree's top levels, four lanes per point operation.
// Below ~2^14 nodes a level is latency-bound: 3 lanes a node, a few waves on
// the whole chip, each lane running two dependent additions of ~14 serial
// Montgomery products (~16 us each).  Here the four lanes of a quad share one
// operation: every round each lane does ONE product (lane-selected operands)
// and the quad exchanges the four results (DPP quad broadcasts), so an
// addition is 4 product rounds deep and a doubling 3, instead of 14 and 8.
// Same formulas as ec29.cuh xadd29 / xdbl29 (squares as mul29: the same
// limbs, tests/test_field29.py), except Y3 = R (Q - X3) + S1 (K - PPP) as
// two products summed (< 2^383) instead of one two-product reduction;
// tests/test_field29.py models both (xadd29w / xdbl29w).
// (masks, not a conditional chain: LLVM turns that into a private array
// indexed by r — 1.3 KB of scratch a lane)
__device__ __forceinline__ F29 qsel(int r, const F29 &a0, const F29 &a1, const F29 &a2, const F29 &a3) {
    const uint32_t m0 = 0u - (uint32_t)(r == 0), m1 = 0u - (uint32_t)(r == 1), m2 = 0u - (uint32_t)(r == 2),
                   m3 = 0u - (uint32_t)(r == 3);
    F29 v;
#pragma unroll
    for (int i = 0; i < 14; i++) v.l[i] = (a0.l[i] & m0) | (a1.l[i] & m1) | (a2.l[i] & m2) | (a3.l[i] & m3);
    return v;
}
// lane S's value to every lane of the quad: a DPP quad_perm broadcast
// [S, S, S, S] (a VALU move; ds_bpermute went through the LDS crossbar)
template <int S>
__device__ __forceinline__ F29 qget(const F29 &v) {
    F29 r;
#pragma unroll
    for (int i = 0; i < 14; i++) r.l[i] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v.l[i], S * 0x55, 0xF, 0xF, false);
    return r;
}
__device__ __forceinline__ F29 add29n(const F29 &a, const F29 &b) {
    F29 r;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 13; i++) {
        const uint32_t t = a.l[i] + b.l[i] + c;
        r.l[i] = t & F29_M;
        c = t >> 29;
    }
    r.l[13] = a.l[13] + b.l[13] + c;
    return r;
}
// p + q on a quad (every lane holds both operands); no exceptional cases
__device__ __forceinline__ Xyzz29 xadd29w(const Xyzz29 &p, const Xyzz29 &q, int r) {
    const F29 m1 = mul29(qsel(r, p.x, q.x, p.y, q.y), qsel(r, q.zz, p.zz, q.zzz, p.zzz));
    const F29 u1 = qget<0>(m1), s1 = qget<2>(m1);
    const F29 P = sub29(qget<1>(m1), u1, F29_KB), R = sub29(qget<3>(m1), s1, F29_KB);
    const F29 m2 = mul29(qsel(r, P, R, p.zz, p.zzz), qsel(r, P, R, q.zz, q.zzz));
    const F29 pp = qget<0>(m2), zzz12 = qget<3>(m2);
    const F29 m3 = mul29(qsel(r, P, u1, qget<2>(m2), P), pp);
    const F29 ppp = qget<0>(m3), qq = qget<1>(m3);
    Xyzz29 o;
    o.zz = qget<2>(m3);
    o.x = sub29(sub29(sub29(qget<1>(m2), ppp, F29_KA), qq, F29_KA), qq, F29_KA);
    const F29 m4 = mul29(qsel(r, zzz12, R, s1, zzz12),
                         qsel(r, ppp, sub29(qq, o.x, F29_KB), neg29(ppp, F29_KA), ppp));
    o.zzz = qget<0>(m4);
    o.y = add29n(qget<1>(m4), qget<2>(m4));
    return o;
}
// 2 p on a quad (dbl-2008-s-1, a = 0)
__device__ __forceinline__ Xyzz29 xdbl29w(const Xyzz29 &p, int r) {
    const F29 U = add29n(p.y, p.y);
    const F29 a1 = qsel(r, U, p.x, U, p.x);
    const F29 m1 = mul29(a1, a1);
    const F29 V = qget<0>(m1), xx = qget<1>(m1);
    const F29 M = add29n(add29n(xx, xx), xx);
    const F29 m2 = mul29(qsel(r, U, p.x, M, V), qsel(r, V, V, M, p.zz));
    const F29 W = qget<0>(m2), S = qget<1>(m2);
    Xyzz29 o;
    o.zz = qget<3>(m2);
    o.x = sub29(sub29(qget<2>(m2), S, F29_KA), S, F29_KA);
    const F29 m3 = mul29(qsel(r, W, M, W, W), qsel(r, p.zzz, sub29(S, o.x, F29_KB), neg29(p.y, F29_KB), p.zzz));
    o.zzz = qget<0>(m3);
    o.y = add29n(qget<1>(m3), qget<2>(m3));
    return o;
}
// the *_inf forms of ec29.cuh; the tests on the operands are the same on the
// four lanes of a quad, so a quad never diverges inside an operation
__device__ __forceinline__ Xyzz29 xadd29w_inf(const Xyzz29 &p, const Xyzz29 &q, int r, uint32_t *exc) {
    if (zero29(p.zz)) return q;
    if (zero29(q.zz)) return p;
    Xyzz29 o = xadd29w(p, q, r);
    if (zero29(o.zz)) *exc = 1u;
    return o;
}
__device__ __forceinline__ Xyzz29 xdbl29w_inf(const Xyzz29 &p, int r) {
    if (zero29(p.zz)) return p;
    return xdbl29w(p, r);
}
// k_tree_level29 with a quad per (node, component); lane r stores coordinate r
__global__ __launch_bounds__(256) void k_tree_level29w(const uint32_t *in, uint64_t nout, uint32_t *out,
                                                       uint32_t *exc) {
    const uint64_t t = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 2;
    if (t >= nout) return;  // whole quads
    const int c = (int)blockIdx.y, r = (int)(threadIdx.x & 3);
    const uint32_t *L = in + 336 * t, *R = L + 168;
    Xyzz29 v;
    if (c == 0) {
        v = xadd29w_inf(load_xyzz29(L), load_xyzz29(R), r, exc);
    } else if (c == 1) {
        v = xadd29w_inf(xadd29w_inf(load_xyzz29(L + 56), load_xyzz29(R + 56), r, exc), load_xyzz29(R + 112), r,
                        exc);
    } else {
        v = xdbl29w_inf(xadd29w_inf(load_xyzz29(L + 112), load_xyzz29(R + 112), r, exc), r);
    }
    store_f29(out + 168 * t + 56 * c + 14 * r, qsel(r, v.x, v.y, v.zz, v.zzz));
}

// k_tree_leafw29 with a quad per leaf (the same running sums and T == S
// tracking; every branch depends on the leaf's buckets only, so a quad stays
// converged): for the small leaf launches of the 8-rank bucket ranges, where
// one lane per leaf is a few waves on the chip
template <int LW>
__global__ __launch_bounds__(256) void k_tree_leafw29w(const uint32_t *bk, const uint32_t *offs, uint64_t nout,
                                                       uint32_t *out, uint32_t *exc) {
    const uint64_t t = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 2;
    if (t >= nout) return;  // whole quads
    const int r = (int)(threadIdx.x & 3);
    const uint64_t u0 = (uint64_t)LW * t;
    Xyzz29 S = bucket29(bk, offs, u0 + LW - 1), T = S;
    bool tis = true;
#pragma unroll 1
    for (int k = LW - 2; k >= 0; k--) {
        const bool empty = offs[u0 + k] == offs[u0 + k + 1];
        if (empty) {
            T = tis ? xdbl29w_inf(T, r) : xadd29w_inf(T, S, r, exc);
            tis = tis && zero29(T.zz);
        } else {
            S = xadd29w_inf(S, load_xyzz29(bk + 56 * (u0 + k)), r, exc);
            const bool tinf = zero29(T.zz);
            T = xadd29w_inf(T, S, r, exc);
            tis = tinf;
        }
    }
    uint32_t *o = out + 168 * t;
    store_f29(o + 14 * r, qsel(r, S.x, S.y, S.zz, S.zzz));
    store_f29(o + 56 + 14 * r, qsel(r, T.x, T.y, T.zz, T.zzz));
    Xyzz29 D = S;
#pragma unroll 1
    for (int k = 1; k < LW; k *= 2) D = xdbl29w_inf(D, r);
    store_f29(o + 112 + 14 * r, qsel(r, D.x, D.y, D.zz, D.zzz));
}

// the roots' T in R384 (the host's 24-u64 XYZZ), then their S (a window's
// plain bucket sum: a bucket-range shard adds lo * S, msm.hip)
__global__ void k_tree_roots29(const uint32_t *in, uint64_t n, uint64_t *out) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (t >= n) return;
    store_xyzz(out + 24 * t, to32(load_xyzz29(in + 168 * t + 56)));
    store_xyzz(out + 24 * (n + t), to32(load_xyzz29(in + 168 * t)));
}

// k_tree_roots29 with a quad per root: lane r converts coordinate r
__global__ void k_tree_roots29w(const uint32_t *in, uint64_t n, uint64_t *out) {
    const uint64_t t = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 2;
    if (t >= n) return;
    const int r = (int)(threadIdx.x & 3);
    store_fq(out + 24 * t + 6 * r, to_fq32(load29(in + 168 * t + 56 + 14 * r)));
    store_fq(out + 24 * (n + t) + 6 * r, to_fq32(load29(in + 168 * t + 14 * r)));
}

const uint64_t *msm_reduce29(const uint32_t *bk29, const uint32_t *offs, uint64_t nwin, int NB,
                             uint32_t *scratch, uint32_t *exc, hipStream_t s) {
    // leaves of PNP_LEAF_W buckets (pairs for the small windows of small MSMs);
    // 4 for the bucket ranges of 8 ranks (NB <= 2^16 a window): there the
    // leaves are latency-bound, a leaf's running sum costs 2 dependent
    // additions per bucket and a tree level 2, so narrower leaves and one more
    // level are shorter — rank 0 of 8 28.6 -> 28.2 ms, one GPU unaffected
    // (its 2^19-bucket windows keep 8; profiles/r06_ab_devseg_leaf.txt)
#ifndef PNP_LEAF_SMALL4
#define PNP_LEAF_SMALL4 1
#endif
    const int LW = NB >= 2 * PNP_LEAF_W ? (PNP_LEAF_SMALL4 && NB <= (1 << 16) && PNP_LEAF_W > 4 ? 4 : PNP_LEAF_W) : 2;
    if (NB < 2 * LW) {
        set_error("msm_reduce29: %d buckets per window", NB);
        throw Error(PNP_E_ARG);
    }
    uint64_t m = nwin * (uint64_t)NB / LW;
    uint32_t *a = scratch, *b = scratch + 168 * m;
    uint64_t *roots = reinterpret_cast<uint64_t *>(scratch + 252 * m);
    const dim3 lgrid((uint32_t)((m + 255) / 256));
    // small leaf launches (the 8-rank ranges' one- and two-MSM batches) on quads
    static const uint64_t leaf_wide = [] {
        const char *e = getenv("PNP_LEAF_WIDE");
        return (uint64_t)(e ? atoll(e) : 32768);
    }();
    const dim3 wgrid((uint32_t)((4 * m + 255) / 256));
    if (LW == 4 && m <= leaf_wide)
        hipLaunchKernelGGL(k_tree_leafw29w<4>, wgrid, dim3(256), 0, s, bk29, offs, m, a, exc);
    else if (LW == 2)
        hipLaunchKernelGGL(k_tree_leafw29<2>, lgrid, dim3(256), 0, s, bk29, offs, m, a, exc);
    else if (LW == 4)
        hipLaunchKernelGGL(k_tree_leafw29<4>, lgrid, dim3(256), 0, s, bk29, offs, m, a, exc);
    else
        hipLaunchKernelGGL(k_tree_leafw29<PNP_LEAF_W>, lgrid, dim3(256), 0, s, bk29, offs, m, a, exc);
    PNP_HIP(hipGetLastError());
    // levels of at most PNP_TREE_WIDE nodes (latency-bound) on quads
    static const uint64_t wide_max = [] {
        const char *e = getenv("PNP_TREE_WIDE");
        return (uint64_t)(e ? atoll(e) : 16384);
    }();
    while (m > nwin) {
        m /= 2;
        if (m <= wide_max)
            hipLaunchKernelGGL(k_tree_level29w, dim3((uint32_t)((4 * m + 255) / 256), 3), dim3(256), 0, s, a, m, b,
                               exc);
        else
            hipLaunchKernelGGL(k_tree_level29, dim3((uint32_t)((m + 255) / 256), 3), dim3(256), 0, s, a, m, b, exc);
        PNP_HIP(hipGetLastError());
        std::swap(a, b);
    }
    hipLaunchKernelGGL(k_tree_roots29w, dim3((uint32_t)((4 * nwin + 255) / 256)), dim3(256), 0, s, a, nwin, roots);
    PNP_HIP(hipGetLastError());
    return roots;
}

// ---------------------------------------------------------------- tree
// the roots' T, packed, then their S
__global__ void k_tree_roots(const uint64_t *in, uint64_t n, uint64_t *out) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (t >= n) return;
    store_xyzz(out + 24 * t, load_xyzz(in + 72 * t + 24));
    store_xyzz(out + 24 * (n + t), load_xyzz(in + 72 * t));
}

const uint64_t *msm_reduce(const uint64_t *bk, uint64_t nwin, int NB, uint64_t *scratch,
                           hipStream_t s) {
    if (NB == 1) return bk;
    // two ping-pong triple arrays: level sizes nwin*NB/2 (or /16), then halving
    const bool wide = NB >= (1 << 18);  // many buckets per window: running-sum leaves
    uint64_t m = nwin * (uint64_t)NB / (wide ? PNP_LEAF_W : 2);
    uint64_t *a = scratch, *b = scratch + 72 * m;
    if (wide)
        hipLaunchKernelGGL(k_tree_leafw<PNP_LEAF_W>, dim3((uint32_t)((m + 255) / 256)), dim3(256), 0, s, bk, m, a);
    else
        hipLaunchKernelGGL(k_tree_leaf, dim3((uint32_t)((m + 255) / 256)), dim3(256), 0, s, bk, m, a);
    PNP_HIP(hipGetLastError());
    while (m > nwin) {
        m /= 2;
        hipLaunchKernelGGL(k_tree_level, dim3((uint32_t)((m + 255) / 256), 3), dim3(256), 0, s, a, m, b);
        PNP_HIP(hipGetLastError());
        std::swap(a, b);
    }
    hipLaunchKernelGGL(k_tree_roots, dim3((uint32_t)((nwin + 255) / 256)), dim3(256), 0, s, a, nwin, b);
    PNP_HIP(hipGetLastError());
    return b;
}

}  // namespace pnp
