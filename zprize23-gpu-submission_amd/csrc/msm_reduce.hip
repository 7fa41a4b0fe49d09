// msm_reduce.hip — Pippenger bucket reduction: sum_b (b+1) B_b per window.
//
// Replaces the reference's per-window running sum on the GPU plus the CPU
// fold (sppark_msm/pippenger.cuh:360-468, zkp/cpu/collect.h:326-489).
//
// Running-sum tree: entry e of a level stands for a contiguous bucket range
// of length `len` (a power of two): T_e = sum_r (r+1) B_r over the range and
// S_e = sum_r B_r.  Groups of G entries merge as T' = sum T_t + len * sum t*S_t;
// the leaves (T = S = B) take the cheaper running-sum form.
//
// These kernels run on few threads (one lane per 8 buckets, then 8x fewer
// per level), so they are latency-bound: this translation unit calls the Fq
// product out of line (PNP_FQ_OUTLINE, ec.cuh), keeping every kernel's hot
// code inside the instruction cache (the inlined XYZZ add is ~150 KB of code;
// a k_reduce with three inlined adds was 1.3 MB and ran at one wave per SIMD).
#define PNP_FQ_OUTLINE 1
#include "msm_internal.h"
#include "ec.cuh"

namespace pnp {

// leaves: 8 buckets -> T = sum (r+1) B_r, S = sum B_r (14 additions)
__global__ __launch_bounds__(256) void k_reduce_leaf(const uint64_t *bk, uint64_t nout,
                                                     uint64_t *outT, uint64_t *outS) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (t >= nout) return;
    Xyzz run = load_xyzz(bk + 24 * (t * 8 + 7));
    Xyzz acc = run;
#pragma unroll 1
    for (int k = 6; k >= 0; k--) {
        run = add(run, load_xyzz(bk + 24 * (t * 8 + k)));
        acc = add(acc, run);
    }
    store_xyzz(outT + 24 * t, acc);
    store_xyzz(outS + 24 * t, run);
}

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
        sumT = add(sumT, load_xyzz(inT + 24 * e));
        run = add(run, load_xyzz(inS + 24 * e));
        if (k > 0) acc = add(acc, run);  // after the loop: acc = sum_{t>=1} t * S_t
    }
#pragma unroll 1
    for (uint32_t d = 0; d < lg_len; d++) acc = dbl(acc);
    store_xyzz(outT + 24 * t, add(sumT, acc));
    store_xyzz(outS + 24 * t, run);
}

const uint64_t *msm_reduce(const uint64_t *bk, uint64_t nwin, int NB, uint64_t *scratch,
                           hipStream_t s) {
    if (NB == 1) return bk;
    uint64_t m = nwin * NB;
    uint64_t per_win = NB;
    uint32_t lg_len = 0;
    const uint64_t *inT = bk, *inS = bk;
    uint64_t *free_ptr = scratch;
    bool leaf = per_win >= 8;
    while (per_win > 1) {
        int G = per_win >= 8 ? 8 : (int)per_win;
        uint64_t nout = m / G;
        uint64_t *oT = free_ptr, *oS = free_ptr + nout * 24;
        free_ptr += 2 * nout * 24;
        uint32_t blocks = (uint32_t)((nout + 255) / 256);
        if (leaf) {
            hipLaunchKernelGGL(k_reduce_leaf, dim3(blocks), dim3(256), 0, s, inT, nout, oT, oS);
            leaf = false;
        } else {
            switch (G) {
                case 8: hipLaunchKernelGGL(k_reduce<8>, dim3(blocks), dim3(256), 0, s, inT, inS, nout, lg_len, oT, oS); break;
                case 4: hipLaunchKernelGGL(k_reduce<4>, dim3(blocks), dim3(256), 0, s, inT, inS, nout, lg_len, oT, oS); break;
                case 2: hipLaunchKernelGGL(k_reduce<2>, dim3(blocks), dim3(256), 0, s, inT, inS, nout, lg_len, oT, oS); break;
                default: set_error("msm reduce: group %d", G); throw Error(PNP_E_ARG);
            }
        }
        PNP_HIP(hipGetLastError());
        inT = oT;
        inS = oS;
        m = nout;
        per_win /= G;
        lg_len += (G == 8 ? 3 : G == 4 ? 2 : 1);
    }
    return inT;
}

}  // namespace pnp
