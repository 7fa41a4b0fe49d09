// msm_internal.h — pieces shared by msm.hip (sort + accumulate) and
// msm_reduce.hip (bucket reduction, compiled with out-of-line Fq products).
#pragma once
#include "pnp_internal.h"

namespace pnp {

// Window geometry for an n-point MSM: c-bit signed digits, W windows,
// NB = 2^(c-1) buckets per window.
struct MsmCfg {
    int c, W, NB;
};

// c = 0: the default for n; W c >= 256 so the top window of a scalar < 2^255
// never carries out of its signed digit
inline MsmCfg msm_cfg(uint64_t n, int c = 0) {
    MsmCfg g;
    int lg = 0;
    while ((1ULL << lg) < n) lg++;
    g.c = lg >= 20 ? 16 : (lg - 3 < 4 ? 4 : lg - 3);
    if (c > 0) g.c = c;
    g.W = (256 + g.c - 1) / g.c;
    g.NB = 1 << (g.c - 1);
    return g;
}

// Buckets split across accumulate lanes (S entries per lane): bucket u whose
// sorted run [offs[u*nch], offs[(u+1)*nch]) spans lanes t0 < t1 is
// tail[t0] + head[t0+1] + ... + head[t1]; empty buckets become infinity.
// `pieces`: typical lanes per bucket (sets the lanes per merge)
void msm_merge_pieces(const uint32_t *offs, int nch, uint64_t U, uint32_t S, uint32_t pieces,
                      const uint64_t *head, const uint64_t *tail, uint64_t *bk, hipStream_t s);

// Sum_b (b+1) * B_b for each of `nwin` consecutive groups of NB XYZZ buckets
// (bk[0 .. nwin*NB), NB a power of two); `scratch` must hold 72*nwin*NB u64.
// Returns the device address of the nwin results (XYZZ, 24 u64 each).

const uint64_t *msm_reduce(const uint64_t *bk, uint64_t nwin, int NB, uint64_t *scratch,
                           hipStream_t s);

}  // namespace pnp
