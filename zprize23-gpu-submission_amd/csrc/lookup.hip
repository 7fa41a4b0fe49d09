// lookup.hip — plookup's sorted multiset on the GPU: MultiSet::combine_split
// (plonk-core/src/lookup/multiset.rs:131-180, called at prover.rs:305-307).
//
// Reference semantics: count every value of t and f, grouped by value, the
// groups in the order of their FIRST occurrence in t (IndexMap insertion
// order); each group of c copies puts floor(c/2) into h1 and h2, and an odd
// group its extra copy into h1 or h2 alternately (h1 first).  Every f value
// must occur in t.  The reference GPU path never runs this (gen_proof.cuh:
// 107-119 hard-codes h1 = h2 = 0 for its f = t = 0 circuit class).
//
// MI355X formulation, no host round trip for the data (one 4-byte error flag):
//   1. the 2n records (t entries tagged 0..n-1 by position, f entries n..2n-1)
//      are sorted by their 256-bit value: four stable LSD passes of hipcub's
//      radix sort on the u64 limbs, payload = the u32 tag.  Stability keeps
//      equal values in tag order, so each run of equal values starts with its
//      first occurrence in t, or with an f tag when the value is not in t;
//   2. run heads -> run ids (inclusive scan); per run: first tag, start;
//   3. runs re-sorted by first tag (the IndexMap order);
//   4. exclusive scans of floor(c/2) and (c & 1) give every run's offset in h1
//      (H + ceil(O/2)) and h2 (H + floor(O/2));
//   5. h1 / h2 filled by output position: a binary search over the run
//      offsets, so a run of n equal padding values costs no more than n runs.
#include <hipcub/hipcub.hpp>
#include "context.h"
#include "protocol.h"

namespace pnp {

namespace {

inline uint32_t nb(uint64_t t, uint32_t bs = 256) { return (uint32_t)((t + bs - 1) / bs); }

__device__ __forceinline__ const uint64_t *rec_value(const uint64_t *t, const uint64_t *f, uint64_t n,
                                                    uint32_t tag) {
    return tag < n ? t + 4 * (uint64_t)tag : f + 4 * ((uint64_t)tag - n);
}

__global__ void k_iota(uint32_t *v, uint64_t m) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < m) v[i] = (uint32_t)i;
}

__global__ void k_limb_keys(const uint64_t *t, const uint64_t *f, uint64_t n, const uint32_t *tags, int limb,
                            uint64_t *keys) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < 2 * n) keys[i] = rec_value(t, f, n, tags[i])[limb];
}

// head[i] = record i starts a run of equal values; an f tag at a head is a
// value absent from t
__global__ void k_heads(const uint64_t *t, const uint64_t *f, uint64_t n, const uint32_t *tags, uint32_t *head,
                        unsigned *err) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= 2 * n) return;
    bool h = i == 0;
    if (!h) {
        const uint64_t *a = rec_value(t, f, n, tags[i]), *b = rec_value(t, f, n, tags[i - 1]);
        h = (a[0] != b[0]) | (a[1] != b[1]) | (a[2] != b[2]) | (a[3] != b[3]);
    }
    head[i] = h;
    if (h && tags[i] >= n) atomicOr(err, 1u);
}

// run r (id = inclusive scan of heads - 1): first tag and start index
__global__ void k_runs(const uint32_t *tags, const uint32_t *head, const uint32_t *rid, uint64_t m,
                       uint32_t *first, uint32_t *start) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= m || !head[i]) return;
    const uint32_t r = rid[i] - 1;
    first[r] = tags[i];
    start[r] = (uint32_t)i;
}

// runs in first-occurrence order: half and odd counts
__global__ void k_run_counts(const uint32_t *order, const uint32_t *start, uint32_t R, uint64_t m,
                             uint32_t *half, uint32_t *odd) {
    uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= R) return;
    const uint32_t r = order[k];
    const uint32_t end = r + 1 < R ? start[r + 1] : (uint32_t)m;
    const uint32_t c = end - start[r];
    half[k] = c >> 1;
    odd[k] = c & 1;
}

// offsets of run k in h1 (even) and h2 (odd): H + ceil(O/2), H + floor(O/2)
__global__ void k_run_offsets(const uint32_t *H, const uint32_t *O, uint32_t R, uint32_t *oe, uint32_t *oo) {
    uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= R) return;
    oe[k] = H[k] + ((O[k] + 1) >> 1);
    oo[k] = H[k] + (O[k] >> 1);
}

// h[p] = value of the last run k with off[k] <= p (off is non-decreasing and
// off[k + 1] = off[k] + copies of run k, so that run has a copy at p)
__global__ void k_fill(const uint64_t *t, const uint64_t *f, uint64_t n, const uint32_t *tags,
                       const uint32_t *order, const uint32_t *start, const uint32_t *off, uint32_t R,
                       uint64_t *h) {
    uint64_t p = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (p >= n) return;
    uint32_t lo = 0, hi = R;  // off[lo] <= p < off[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (off[mid] <= p) lo = mid; else hi = mid;
    }
    const uint64_t *v = rec_value(t, f, n, tags[start[order[lo]]]);
    reinterpret_cast<ulonglong2 *>(h + 4 * p)[0] = make_ulonglong2(v[0], v[1]);
    reinterpret_cast<ulonglong2 *>(h + 4 * p)[1] = make_ulonglong2(v[2], v[3]);
}

}  // namespace

bool combine_split(pnp_ctx *ctx, const uint64_t *t, const uint64_t *f, uint64_t n, uint64_t *h1,
                   uint64_t *h2, hipStream_t s) {
    const uint64_t m = 2 * n;
    if (m >= (1ULL << 32)) {
        set_error("combine_split: %llu entries exceed the u32 tags", (unsigned long long)m);
        throw Error(PNP_E_ARG);
    }
    // u32 scratch carved from named work buffers (sized in 32-byte units)
    auto u32buf = [&](const char *name, uint64_t cnt) {
        return reinterpret_cast<uint32_t *>(ctx->buf(name, (cnt * 4 + 31) / 32 + 1));
    };
    uint32_t *tag_a = u32buf("cs_tag_a", m), *tag_b = u32buf("cs_tag_b", m);
    uint32_t *head = u32buf("cs_head", m), *rid = u32buf("cs_rid", m);
    uint64_t *key_a = ctx->buf("cs_key_a", (m * 8 + 31) / 32), *key_b = ctx->buf("cs_key_b", (m * 8 + 31) / 32);
    uint32_t *first = u32buf("cs_first", m), *start = u32buf("cs_start", m);
    uint32_t *first_s = u32buf("cs_first_s", m), *order_in = u32buf("cs_order_in", m);
    uint32_t *order = u32buf("cs_order", m);
    uint32_t *half = u32buf("cs_half", m), *odd = u32buf("cs_odd", m);
    uint32_t *H = u32buf("cs_H", m), *O = u32buf("cs_O", m), *oe = u32buf("cs_oe", m), *oo = u32buf("cs_oo", m);
    unsigned *err = u32buf("cs_err", 4);
    PNP_HIP(hipMemsetAsync(err, 0, 4, s));

    // temporary storage for the hipcub passes (the largest of them)
    size_t tmp_bytes = 0, b = 0;
    PNP_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, b, key_a, key_b, tag_a, tag_b, (int)m, 0, 64, s));
    tmp_bytes = std::max(tmp_bytes, b);
    PNP_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, b, first, first_s, order_in, order, (int)m, 0, 32, s));
    tmp_bytes = std::max(tmp_bytes, b);
    PNP_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, b, head, rid, (int)m, s));
    tmp_bytes = std::max(tmp_bytes, b);
    PNP_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, b, half, H, (int)m, s));
    tmp_bytes = std::max(tmp_bytes, b);
    void *tmp = ctx->buf("cs_tmp", tmp_bytes / 32 + 1);

    // 1. stable LSD sort of the records by value
    hipLaunchKernelGGL(k_iota, dim3(nb(m)), dim3(256), 0, s, tag_a, m);
    for (int limb = 0; limb < 4; limb++) {
        hipLaunchKernelGGL(k_limb_keys, dim3(nb(m)), dim3(256), 0, s, t, f, n, tag_a, limb, key_a);
        PNP_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, key_a, key_b, tag_a, tag_b, (int)m, 0, 64, s));
        std::swap(tag_a, tag_b);
    }
    // 2. runs
    hipLaunchKernelGGL(k_heads, dim3(nb(m)), dim3(256), 0, s, t, f, n, tag_a, head, err);
    PNP_HIP(hipcub::DeviceScan::InclusiveSum(tmp, tmp_bytes, head, rid, (int)m, s));
    uint32_t R = 0;
    unsigned herr = 0;
    PNP_HIP(hipMemcpyAsync(&R, rid + m - 1, 4, hipMemcpyDeviceToHost, s));
    PNP_HIP(hipMemcpyAsync(&herr, err, 4, hipMemcpyDeviceToHost, s));
    PNP_HIP(hipStreamSynchronize(s));
    if (herr) return false;
    hipLaunchKernelGGL(k_runs, dim3(nb(m)), dim3(256), 0, s, tag_a, head, rid, m, first, start);
    // 3. runs in the order of their first occurrence in t
    hipLaunchKernelGGL(k_iota, dim3(nb(R)), dim3(256), 0, s, order_in, (uint64_t)R);
    PNP_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, first, first_s, order_in, order, (int)R, 0, 32, s));
    // 4. offsets in h1 / h2
    hipLaunchKernelGGL(k_run_counts, dim3(nb(R)), dim3(256), 0, s, order, start, R, m, half, odd);
    PNP_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, half, H, (int)R, s));
    PNP_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, odd, O, (int)R, s));
    hipLaunchKernelGGL(k_run_offsets, dim3(nb(R)), dim3(256), 0, s, H, O, R, oe, oo);
    // 5. fill
    hipLaunchKernelGGL(k_fill, dim3(nb(n)), dim3(256), 0, s, t, f, n, tag_a, order, start, oe, R, h1);
    hipLaunchKernelGGL(k_fill, dim3(nb(n)), dim3(256), 0, s, t, f, n, tag_a, order, start, oo, R, h2);
    PNP_HIP(hipGetLastError());
    return true;
}

}  // namespace pnp
