// msm_internal.h — pieces shared by msm.hip (sort + accumulate) and
// msm_reduce.hip (bucket reduction, compiled with out-of-line Fq products).
#pragma once
#include "pnp_internal.h"

namespace pnp {

// Window geometry for an n-point MSM: c-bit signed digits, W windows,
// NB = 2^(c-1) buckets per window.
struct MsmCfg {
    int c, W, NB;
    // folded tables: the top window's digit d is taken as bucket d 2^top_sh
    // against table level W-1 = 2^(c (W-1) - top_sh) P (msm_build_table).  A
    // scalar < 2^255 leaves only 255 - c (W-1) bits (+ a carry) for the top
    // window (15 of c = 20): unscaled, its entries — one per point and MSM —
    // would all land in the lowest 2^15 of the 2^19 buckets, 2.3x their share,
    // and in a bucket-range sharded MSM on rank 0 alone (1.67x the entries of
    // the other ranks at 8 GPUs); scaled they spread over every bucket range
    int top_sh;
};

// c = 0: the default for n; W c >= 256 so the top window of a scalar < 2^255
// never carries out of its signed digit.  folded: the fixed-base layout (one
// bucket set per MSM, cheap to reduce) takes wider windows — c = 20 gives 13
// windows instead of 16 (measured -16% accumulation, -7% per proof at 2^22).
inline MsmCfg msm_cfg(uint64_t n, int c = 0, bool folded = false) {
    MsmCfg g;
    int lg = 0;
    while ((1ULL << lg) < n) lg++;
    // folded: c = 20 from 2^19 points (one rank's range of an 8-GPU proof at
    // n = 2^22): measured per MSM at 2^19 / 2^20 / 2^21 points, c = 20 beats
    // 16..19 (tools/msm_c_sweep.sh, profiles/r02_msm_c_sweep.jsonl)
    if (folded)
        g.c = lg >= 19 ? 20 : (lg - 3 < 4 ? 4 : lg - 3);
    else
        g.c = lg >= 20 ? 16 : (lg - 3 < 4 ? 4 : lg - 3);
    if (c > 0) g.c = c;
    g.W = (256 + g.c - 1) / g.c;
    g.NB = 1 << (g.c - 1);
    const int top_bits = 255 - g.c * (g.W - 1);  // top raw value <= 2^top_bits (carry included)
    g.top_sh = folded && top_bits >= 0 && g.c - 1 - top_bits > 0 ? g.c - 1 - top_bits : 0;
    return g;
}

// Buckets split across accumulate lanes (S entries per lane): bucket u whose
// sorted run [offs[u*nch], offs[(u+1)*nch]) spans lanes t0 < t1 is
// tail[t0] + head[t0+1] + ... + head[t1]; empty buckets become infinity.
// `pieces`: typical lanes per bucket (sets the lanes per merge)
void msm_merge_pieces(const uint32_t *offs, int nch, uint64_t U, uint32_t S, uint32_t pieces,
                      const uint64_t *head, const uint64_t *tail, uint64_t *bk, hipStream_t s);

// the same over raw radix-2^29 pieces (folded layout, 56 u32 each, ec29.cuh),
// one merge lane per accumulation lane t whose segment ended inside bucket
// tailb[t] (NO_TAIL otherwise; tlist: [0] the count, then those lanes t,
// compacted by the accumulation): bk29 holds the buckets inside one lane's
// segment on entry and every NON-EMPTY bucket (F29) on exit; empty buckets
// (offs[u] = offs[u + 1]) are left unwritten and read as infinity by
// msm_reduce29.  (An equal / opposite pair of operands sets *exc: see
// msm_reduce29.)  `heavy`: U + 1 u32 of scratch (count, then the queued
// buckets of > 64 pieces).
constexpr uint32_t NO_TAIL = 0xFFFFFFFFu;

// Segment length of an accumulation launch.  The host sizes the launch (nthr
// lanes of S entries, whole rounds of the chip's wave slots) from an upper
// bound of the sorted entries — MSMs x windows x points, or the fixed slots'
// capacity — before the sort has counted them; zero digits, copy groups and
// padding rows drop out, so a launch can hold far fewer (round 1's wires: 82 M
// of 218 M), and lanes of S entries then leave part of the chip idle (a round
// 0.74 full at rank 0 of 8).  PNP_ACC_DEVSEG=1: every kernel that walks the
// segments takes S = ceil(total / nthr) from the device count instead (never
// above the host's S, at least 16), so the launch's lanes share the real
// entries evenly; all of them compute the same S from offs[U].  Measured
// (same box, 3 interleaved rounds, profiles/r06_ab_devseg_leaf.txt): one GPU
// 0.1284 -> 0.1299 s (the shorter segments split more buckets: more pieces
// to store and merge), rank 0 of 8 neutral (28.5 vs 28.6 ms) — off
#ifndef PNP_ACC_DEVSEG
#define PNP_ACC_DEVSEG 0
#endif
__device__ __forceinline__ uint32_t acc_seg(const uint32_t *offs, uint64_t U, uint64_t nthr, uint32_t S) {
#if PNP_ACC_DEVSEG
    const uint64_t total = offs[U];
    uint64_t d = (total + nthr - 1) / nthr;
    d = d < 16 ? 16 : d;
    return d < S ? (uint32_t)d : S;
#else
    (void)offs, (void)U, (void)nthr;
    return S;
#endif
}
void msm_merge_pieces29(const uint32_t *offs, uint64_t U, uint32_t S, uint64_t nthr, const uint32_t *tailb,
                        const uint32_t *tlist, uint32_t *bk29, const uint32_t *head, const uint32_t *tail, uint32_t *exc,
                        uint32_t *heavy, hipStream_t s);
// exact fallback: the same pieces summed in 32-bit Fq into bk (R384)
void msm_merge_pieces29_exact(const uint32_t *offs, uint64_t U, uint32_t S, uint64_t nthr, uint32_t pieces,
                              const uint32_t *bk29, const uint32_t *head, const uint32_t *tail, uint64_t *bk,
                              hipStream_t s);

// Sum_b (b+1) * B_b for each of `nwin` consecutive groups of NB XYZZ buckets
// (bk[0 .. nwin*NB), NB a power of two); `scratch` must hold 72*nwin*NB u64.
// Returns the device address of the nwin results (XYZZ, 24 u64 each),
// followed by the nwin plain sums Sum_b B_b.

const uint64_t *msm_reduce(const uint64_t *bk, uint64_t nwin, int NB, uint64_t *scratch,
                           hipStream_t s);
// the same over radix-2^29 buckets (56 u32 each); `scratch` must hold
// 126 * nwin * NB + 96 * nwin u32 (NB >= 4); results R384 (T, then S).  *exc is set when
// an addition met equal or opposite operands (never for random inputs): the
// results are then wrong and the caller redoes the group with
// msm_merge_pieces29_exact + msm_reduce (32-bit, exact)
// `offs`: the nwin*NB + 1 bucket starts (empty buckets are infinity whatever
// bk29 holds for them)
const uint64_t *msm_reduce29(const uint32_t *bk29, const uint32_t *offs, uint64_t nwin, int NB,
                             uint32_t *scratch, uint32_t *exc, hipStream_t s);

}  // namespace pnp
