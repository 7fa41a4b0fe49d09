// Batch-affine bucket accumulation, measured.
//
// One pairwise-tree level of a folded MSM in affine coordinates with a shared
// inversion (Montgomery's trick), against the XYZZ mixed addition the
// production kernel (msm.hip k_accumulate29) does, on the same box, the same
// table layout (x, y radix 2^29, R = 2^406, one 128-B line per point) and the
// same number of random gathers:
//   pass 1  (k_ba_prefix): lane l owns pairs p = k L + l, k < K; gathers the
//           two points' x (the first 64 B of each line), d = x2 - x1, running
//           product P_k = d_0 ... d_k, stores P_0 .. P_(K-2) (56 B each,
//           coalesced over the lanes) and the lane total P_(K-1);
//   inverse (k_ba_inv_lvl2): the lane totals inverted by a second Montgomery
//           level (64 totals a lane, prefix, one Fermat inversion, back pass):
//           ~3 products per total plus 1/64 of an inversion;
//   pass 2  (k_ba_finish): back over the lane's pairs: 1/d_k = inv P_(k-1),
//           inv *= d_k, lambda = (y2 - y1) / d_k, x3 = lambda^2 - x1 - x2,
//           y3 = lambda (x1 - x3) - y1 (gathers both lines again, writes the
//           128-B result line).
//   Products per addition: 1 + 2 + 3 = 6 (5 mul + 1 sqr) against XYZZ's
//   8 mul + 2 sqr (9 reductions with the paired y3 product).
// Baseline (k_xyzz_chain): every lane sums 2K gathered points of the same
// random index stream into one XYZZ accumulator (madd-2008-s, exactly
// msm.hip madd29), register-prefetching the next point.
//
// Values are random field elements below 2^383, not curve points: the
// formulas, bounds and memory traffic are what is timed.  The first pairs'
// inputs and outputs are written to a file checked in Python
// (tools/ubench_batch_affine_check.py: the affine formulas mod q).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I zprize23-gpu-submission_amd/csrc \
//       tools/ubench_batch_affine.hip -o tools/ubench_batch_affine
//   ./tools/ubench_batch_affine [lg_pairs=26] [check_file]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include "ec29.cuh"
using namespace pnp;

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

constexpr uint64_t PT = 32;  // u32 per table point (x, y, padding: one 128-B line)
// u32 per F29 in the prefix / total / scratch arrays: 64 B, so every element is
// 16-B aligned (load29's 8-byte tail load is widened to 16 bytes by the
// compiler on that assumption: at a 56-B stride the last element's widened load
// crossed the end of the allocation and faulted)
constexpr uint64_t SF = 16;

// bounds of every array the batch-affine kernels index (checked per access:
// an index out of range is counted in *bad and clamped, never dereferenced)
struct Lim {
    uint64_t tab_pts, pairs, pre_elems, tot_elems, out_pts;
    uint32_t *bad;
};
__device__ __forceinline__ uint64_t chk(uint64_t i, uint64_t n, const Lim &lim) {
    if (i >= n) {
        atomicAdd(lim.bad, 1u);
        return 0;
    }
    return i;
}

__device__ __forceinline__ F29 ld29(const uint32_t *p) { return load29(p); }
__device__ __forceinline__ F29 ld29_x_half(const uint32_t *p) {
    // x = the first 14 words of the line (3 x 16 B + 8 B: inside its first 64 B)
    return load29(p);
}

// madd-2008-s (as msm.hip madd29): P += (x2, y2)
__device__ __forceinline__ void madd29_ub(Xyzz29 &p, const F29 &x2, const F29 &y2) {
    F29 u2 = mul29(x2, p.zz);
    F29 s2 = mul29(y2, p.zzz);
    F29 P = sub29(u2, p.x, F29_KB);
    F29 R = sub29(s2, p.y, F29_KB);
    F29 pp = sqr29(P);
    F29 ppp = mul29(P, pp);
    F29 q = mul29(p.x, pp);
    F29 x3 = sub29(sub29(sub29(sqr29(R), ppp, F29_KA), q, F29_KA), q, F29_KA);
    F29 y3 = mul2_29(R, sub29(q, x3, F29_KB), p.y, neg29(ppp, F29_KA));
    p.zz = mul29(p.zz, pp);
    p.zzz = mul29(p.zzz, ppp);
    p.x = x3;
    p.y = y3;
}

// PF: the next point prefetched into registers (3 waves per SIMD, some
// spilling) or loaded at the top of the iteration (4 waves per SIMD, the
// other waves' products hide the gather)
template <bool PF>
__global__ __launch_bounds__(256, PF ? 3 : 4) void k_xyzz_chain(const uint32_t *tab, const uint32_t *idx,
                                                                 uint64_t L, int K2, uint32_t *out) {
    const uint64_t l = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (l >= L) return;
    Xyzz29 acc;
    const uint32_t *p0 = tab + PT * idx[l];
    acc.x = ld29(p0);
    acc.y = ld29(p0 + 14);
    acc.zz = const29(F29_ONE);
    acc.zzz = const29(F29_ONE);
    F29 nx, ny;
    if (PF) {
        const uint32_t *pn = tab + PT * idx[L + l];
        nx = ld29(pn);
        ny = ld29(pn + 14);
    }
#pragma unroll 1
    for (int k = 1; k < K2; k++) {
        F29 x, y;
        if (PF) {
            x = nx, y = ny;
            if (k + 1 < K2) {
                const uint32_t *q = tab + PT * idx[(uint64_t)(k + 1) * L + l];
                nx = ld29(q);
                ny = ld29(q + 14);
            }
        } else {
            const uint32_t *q = tab + PT * idx[(uint64_t)k * L + l];
            x = ld29(q);
            y = ld29(q + 14);
        }
        madd29_ub(acc, x, y);
    }
    store_xyzz29(out + 56 * l, acc);
}

// pass 1: running products of d = x2 - x1 over the lane's K pairs
__global__ __launch_bounds__(256) void k_ba_prefix(const uint32_t *tab, const uint2 *pairs, uint64_t L, int K,
                                                    uint32_t *prefix, uint32_t *total, Lim lim) {
    const uint64_t l = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (l >= L) return;
    F29 acc;
    uint2 e = pairs[chk(l, lim.pairs, lim)];
    F29 nx1 = ld29_x_half(tab + PT * chk(e.x, lim.tab_pts, lim)), nx2 = ld29_x_half(tab + PT * chk(e.y, lim.tab_pts, lim));
#pragma unroll 1
    for (int k = 0; k < K; k++) {
        const F29 x1 = nx1, x2 = nx2;
        if (k + 1 < K) {
            e = pairs[chk((uint64_t)(k + 1) * L + l, lim.pairs, lim)];
            nx1 = ld29_x_half(tab + PT * chk(e.x, lim.tab_pts, lim));
            nx2 = ld29_x_half(tab + PT * chk(e.y, lim.tab_pts, lim));
        }
        const F29 d = sub29(x2, x1, F29_KB);
        acc = k ? mul29(acc, d) : d;
        if (k + 1 < K) store_f29(prefix + SF * chk((uint64_t)k * L + l, lim.pre_elems, lim), acc);
    }
    store_f29(total + SF * chk(l, lim.tot_elems, lim), acc);
}

// a^(q-2) in the Montgomery form (R = 2^406): the Montgomery form of a^-1
__device__ F29 inv29_fermat(const F29 &a) {
    // q - 2, 381 bits, most significant first (F29_QM2 words, little-endian u32)
    constexpr uint32_t E[12] = {0xffffaaa9u, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u,
                                0xf38512bfu, 0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau};
    F29 r = a;
    for (int b = 379; b >= 0; b--) {  // bit 380 (the top) is the start value
        r = sqr29(r);
        if ((E[b >> 5] >> (b & 31)) & 1) r = mul29(r, a);
    }
    return r;
}

// the lane totals (L of them) inverted: lanes of 64 totals (strided), prefix,
// one Fermat inversion, back pass
__global__ __launch_bounds__(256) void k_ba_inv_lvl2(uint32_t *total, uint64_t L, uint32_t *scratch, Lim lim) {
    const uint64_t L2 = (L + 63) / 64;
    const uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (j >= L2) return;
    F29 acc;
    int cnt = 0;
    for (uint64_t i = j; i < L; i += L2, cnt++) {
        const F29 t = ld29(total + SF * chk(i, lim.tot_elems, lim));
        acc = cnt ? mul29(acc, t) : t;
        store_f29(scratch + SF * chk(i, lim.tot_elems, lim), acc);
    }
    if (!cnt) return;
    F29 inv = inv29_fermat(acc);
    for (int c = cnt - 1; c >= 0; c--) {
        const uint64_t i = j + (uint64_t)c * L2;
        const F29 t = ld29(total + SF * chk(i, lim.tot_elems, lim));
        const F29 ti = c ? mul29(inv, ld29(scratch + SF * chk(i - L2, lim.tot_elems, lim))) : inv;
        if (c) inv = mul29(inv, t);
        store_f29(total + SF * chk(i, lim.tot_elems, lim), ti);  // total[i] <- total[i]^-1
    }
}

// pass 2: back over the pairs, finishing every affine addition (PF as above)
template <bool PF>
__global__ __launch_bounds__(256, PF ? 3 : 4) void k_ba_finish(const uint32_t *tab, const uint2 *pairs, uint64_t L,
                                                                int K, const uint32_t *prefix,
                                                                const uint32_t *total_inv, uint32_t *out, Lim lim) {
    const uint64_t l = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (l >= L) return;
    F29 inv = ld29(total_inv + SF * chk(l, lim.tot_elems, lim));
    F29 nx1, ny1, nx2, ny2;
    auto gather = [&](int k, F29 &x1, F29 &y1, F29 &x2, F29 &y2) {
        const uint2 e = pairs[chk((uint64_t)k * L + l, lim.pairs, lim)];
        const uint32_t *a = tab + PT * chk(e.x, lim.tab_pts, lim), *b = tab + PT * chk(e.y, lim.tab_pts, lim);
        x1 = ld29(a), y1 = ld29(a + 14), x2 = ld29(b), y2 = ld29(b + 14);
    };
    if (PF) gather(K - 1, nx1, ny1, nx2, ny2);
#pragma unroll 1
    for (int k = K - 1; k >= 0; k--) {
        F29 x1, y1, x2, y2;
        if (PF) {
            x1 = nx1, y1 = ny1, x2 = nx2, y2 = ny2;
            if (k) gather(k - 1, nx1, ny1, nx2, ny2);
        } else {
            gather(k, x1, y1, x2, y2);
        }
        const F29 d = sub29(x2, x1, F29_KB);
        F29 di = inv;
        if (k) {
            const F29 pk = ld29(prefix + SF * chk((uint64_t)(k - 1) * L + l, lim.pre_elems, lim));
            di = mul29(inv, pk);
            inv = mul29(inv, d);
        }
        const F29 lam = mul29(sub29(y2, y1, F29_KB), di);
        const F29 x3 = sub29(sub29(sqr29(lam), x1, F29_KA), x2, F29_KA);
        const F29 y3 = sub29(mul29(lam, sub29(x1, x3, F29_KB)), y1, F29_KA);
        uint32_t *o = out + PT * chk((uint64_t)k * L + l, lim.out_pts, lim);
        store_f29(o, x3);
        store_f29(o + 14, y3);
    }
}

static uint64_t rs = 88172645463325252ULL;
static inline uint64_t rnd() {
    rs ^= rs << 13;
    rs ^= rs >> 7;
    rs ^= rs << 17;
    return rs;
}

int main(int argc, char **argv) {
    const int lgp = argc > 1 ? atoi(argv[1]) : 26;
    const char *check = argc > 2 ? argv[2] : nullptr;
    const uint64_t P = 1ULL << lgp;           // pairs = additions of the level
    const uint64_t T = 13ULL << 22;           // table points: the 2^22 folded table's 13 windows
    // table: random limbs, value < 2^383 (top limb < 2^6)
    std::vector<uint32_t> h(T * PT);
    for (uint64_t i = 0; i < T; i++) {
        for (int w = 0; w < 28; w++) h[PT * i + w] = (uint32_t)rnd() & F29_M;
        h[PT * i + 13] &= 0x3F;
        h[PT * i + 27] &= 0x3F;
        for (int w = 28; w < 32; w++) h[PT * i + w] = 0;
    }
    std::vector<uint32_t> hi(2 * P);
    for (auto &v : hi) v = (uint32_t)(rnd() % T);
    uint32_t *tab, *idx, *pre, *tot, *scr, *out, *xo;
    CK(hipMalloc(&tab, h.size() * 4 + 256));
    CK(hipMalloc(&idx, hi.size() * 4 + 256));
    CK(hipMemcpy(tab, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(idx, hi.data(), hi.size() * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&pre, P * SF * 4 + 256));
    CK(hipMalloc(&out, P * 128 + 256));
    uint32_t *bad;
    CK(hipMalloc(&bad, 4));
    CK(hipMemset(bad, 0, 4));
    hipEvent_t e0, e1, e2, e3;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&e2));
    CK(hipEventCreate(&e3));
    printf("batch-affine vs XYZZ, one pairwise level: %llu additions (2^%d), table %llu points x 128 B\n",
           (unsigned long long)P, lgp, (unsigned long long)T);
    // XYZZ baseline: 2K points a lane -> 2K - 1 madds; L2 lanes
    for (int K2 : {32, 64, 128})
    for (int pf = 0; pf < 2; pf++) {
        const uint64_t L2 = 2 * P / K2;
        CK(hipMalloc(&xo, L2 * 224 + 256));
        float best = 1e30f;
        for (int rep = 0; rep < 3; rep++) {
            CK(hipEventRecord(e0));
            if (pf)
                hipLaunchKernelGGL(k_xyzz_chain<true>, dim3((uint32_t)((L2 + 255) / 256)), dim3(256), 0, 0, tab, idx,
                                   L2, K2, xo);
            else
                hipLaunchKernelGGL(k_xyzz_chain<false>, dim3((uint32_t)((L2 + 255) / 256)), dim3(256), 0, 0, tab, idx,
                                   L2, K2, xo);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        const double adds = (double)L2 * (K2 - 1);
        printf("XYZZ chain  K2=%3d prefetch=%d: %8.3f ms, %.1f ps per madd, %.0f B gathered per madd "
               "(one line per entry)\n", K2, pf, best, 1e9 * best / adds, 128.0 * 2 * P / adds);
        CK(hipFree(xo));
    }
    for (int K : {16, 32, 64, 128})
    for (int pf = 0; pf < 2; pf++) {
        const uint64_t L = P / K;
        CK(hipMalloc(&tot, L * SF * 4 + 256));
        CK(hipMalloc(&scr, L * SF * 4 + 256));
        const Lim lim{T, P, P, L, P, bad};
        float b1 = 1e30f, b2 = 1e30f, b3 = 1e30f;
        for (int rep = 0; rep < 3; rep++) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_ba_prefix, dim3((uint32_t)((L + 255) / 256)), dim3(256), 0, 0, tab,
                               reinterpret_cast<const uint2 *>(idx), L, K, pre, tot, lim);
            CK(hipEventRecord(e1));
            if (rep == 0) {  // (the first round synchronises after every kernel: a fault names its kernel)
                CK(hipEventSynchronize(e1));
                fprintf(stderr, "K=%d pf=%d prefix ok\n", K, pf);
            }
            const uint64_t L2 = (L + 63) / 64;
            hipLaunchKernelGGL(k_ba_inv_lvl2, dim3((uint32_t)((L2 + 255) / 256)), dim3(256), 0, 0, tot, L, scr, lim);
            CK(hipEventRecord(e2));
            if (rep == 0) {
                CK(hipEventSynchronize(e2));
                fprintf(stderr, "K=%d pf=%d inverse ok\n", K, pf);
            }
            if (pf)
                hipLaunchKernelGGL(k_ba_finish<true>, dim3((uint32_t)((L + 255) / 256)), dim3(256), 0, 0, tab,
                                   reinterpret_cast<const uint2 *>(idx), L, K, pre, tot, out, lim);
            else
                hipLaunchKernelGGL(k_ba_finish<false>, dim3((uint32_t)((L + 255) / 256)), dim3(256), 0, 0, tab,
                                   reinterpret_cast<const uint2 *>(idx), L, K, pre, tot, out, lim);
            CK(hipEventRecord(e3));
            CK(hipEventSynchronize(e3));
            float m1, m2, m3;
            CK(hipEventElapsedTime(&m1, e0, e1));
            CK(hipEventElapsedTime(&m2, e1, e2));
            CK(hipEventElapsedTime(&m3, e2, e3));
            if (m1 + m2 + m3 < b1 + b2 + b3) b1 = m1, b2 = m2, b3 = m3;
        }
        CK(hipGetLastError());
        uint32_t nbad = 0;
        CK(hipMemcpy(&nbad, bad, 4, hipMemcpyDeviceToHost));
        if (nbad) {
            printf("batch-affine K=%d: %u out-of-range indices (clamped, not dereferenced)\n", K, nbad);
            return 2;
        }
        const double tot_ms = b1 + b2 + b3;
        // bytes per addition as laid out here: pass 1: 8 B pair + 2 x 64 B x halves + 64 B prefix
        // (K-1 of K); pass 2: 8 B + 2 x 128 B lines + 64 B prefix + 128 B out; the totals' level
        // ~ 4 x 64 / K
        const double bytes = 8 + 128 + 64.0 * (K - 1) / K + 8 + 256 + 64.0 * (K - 1) / K + 128 + 4 * 64.0 / K;
        printf("batch-affine K=%3d prefetch=%d: %8.3f ms (prefix %.3f, inverse %.3f, finish %.3f), %.1f ps per addition, "
               "%.0f B per addition (%.2f TB/s)\n",
               K, pf, tot_ms, b1, b2, b3, 1e9 * tot_ms / P, bytes, bytes * P / (tot_ms * 1e-3) / 1e12);
        if (check && K == 64 && pf == 0) {
            // first 4 pairs of lane 0..3 at k = 0: inputs and outputs
            FILE *f = fopen(check, "w");
            std::vector<uint32_t> o(PT * 4);
            CK(hipMemcpy(o.data(), out, o.size() * 4, hipMemcpyDeviceToHost));
            fprintf(f, "[\n");
            for (int p = 0; p < 4; p++) {
                const uint32_t a = hi[2 * p], b = hi[2 * p + 1];
                auto dump = [&](const uint32_t *v) {
                    fprintf(f, "[");
                    for (int w = 0; w < 14; w++) fprintf(f, "%u%s", v[w], w < 13 ? "," : "");
                    fprintf(f, "]");
                };
                fprintf(f, " {\"x1\": ");
                dump(&h[PT * a]);
                fprintf(f, ", \"y1\": ");
                dump(&h[PT * a + 14]);
                fprintf(f, ", \"x2\": ");
                dump(&h[PT * b]);
                fprintf(f, ", \"y2\": ");
                dump(&h[PT * b + 14]);
                fprintf(f, ", \"x3\": ");
                dump(&o[PT * p]);
                fprintf(f, ", \"y3\": ");
                dump(&o[PT * p + 14]);
                fprintf(f, "}%s\n", p < 3 ? "," : "");
            }
            fprintf(f, "]\n");
            fclose(f);
        }
        CK(hipFree(tot));
        CK(hipFree(scr));
    }
    return 0;
}
