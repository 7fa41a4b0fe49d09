// A/B of the Karatsuba a*b half (field29.cuh mul29k / mul2_29k) against the
// schoolbook radix-2^29 Montgomery product (mul29 / mul2_29), inside the MSM
// bucket loop's mixed addition (msm.hip madd29) over randomly gathered points
// of a 512 MiB table, and on independent products.  Both variants compute the
// same integers (same columns, same Montgomery quotients): the checksums must
// agree.  Prints Gmadd/s, Gmul/s and VGPRs per variant.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../zprize23-gpu-submission_amd/csrc ubench_kara.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include "field29.cuh"
#include "ec29.cuh"
using namespace pnp;

template <bool K>
__device__ __forceinline__ F29 MUL(const F29 &a, const F29 &b) {
    if constexpr (K) return mul29k(a, b); else return mul29(a, b);
}
template <bool K>
__device__ __forceinline__ F29 MUL2(const F29 &a, const F29 &b, const F29 &c, const F29 &d) {
    if constexpr (K) return mul2_29k(a, b, c, d); else return mul2_29(a, b, c, d);
}

// msm.hip madd29 with the product chosen by K
template <bool K>
__device__ __forceinline__ void madd(Xyzz29 &p, const F29 &x2, const F29 &y2) {
    F29 u2 = MUL<K>(x2, p.zz);
    F29 s2 = MUL<K>(y2, p.zzz);
    F29 P = sub29(u2, p.x, F29_KB);
    F29 R = sub29(s2, p.y, F29_KB);
    F29 pp = sqr29(P);
    F29 ppp = MUL<K>(P, pp);
    F29 q = MUL<K>(p.x, pp);
    F29 x3 = sub29(sub29(sub29(sqr29(R), ppp, F29_KA), q, F29_KA), q, F29_KA);
    F29 y3 = MUL2<K>(R, sub29(q, x3, F29_KB), p.y, neg29(ppp, F29_KA));
    p.zz = MUL<K>(p.zz, pp);
    p.zzz = MUL<K>(p.zzz, ppp);
    p.x = x3;
    p.y = y3;
}

template <bool K>
__global__ __launch_bounds__(256, 3) void k_madd(const uint32_t *pts, uint64_t npts, int L, uint32_t *out) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t h = (t + 1) * 0x9E3779B97F4A7C15ULL;
    Xyzz29 acc;
    acc.x = load29(pts + 32 * (t % npts));
    acc.y = load29(pts + 32 * (t % npts) + 14);
    acc.zz = acc.zzz = const29(F29_ONE);
#pragma unroll 1
    for (int i = 0; i < L; i++) {
        h = h * 6364136223846793005ULL + 1442695040888963407ULL;
        const uint32_t *p = pts + 32 * ((h >> 24) % npts);
        F29 x = load29(p), y = load29(p + 14);
        if (h & 1) y = neg29(y, F29_KA);
        madd<K>(acc, x, y);
    }
    store_xyzz29(out + 56 * t, acc);
}

template <bool K>
__global__ __launch_bounds__(256, 3) void k_mul(const uint32_t *pts, int L, uint32_t *out) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    F29 a = load29(pts + 32 * (t & 1023)), b = load29(pts + 32 * ((t + 1) & 1023) + 14);
    F29 c = a, d = b;
#pragma unroll 1
    for (int i = 0; i < L; i++) {  // 4 independent products per iteration
        a = MUL<K>(a, b); c = MUL<K>(c, d); b = MUL<K>(b, c); d = MUL<K>(d, a);
    }
    store_f29(out + 56 * t, a);
    store_f29(out + 56 * t + 14, b);
    store_f29(out + 56 * t + 28, c);
    store_f29(out + 56 * t + 42, d);
}

// random field elements < q in radix 2^29 (R406 form is irrelevant here:
// any values < 2q are valid product inputs)
static void fill(std::vector<uint32_t> &v, uint64_t n) {
    uint64_t s = 88172645463325252ULL;
    auto rnd = [&] { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
    v.assign(32 * n, 0);
    for (uint64_t i = 0; i < n; i++)
        for (int c = 0; c < 2; c++) {
            uint32_t *l = &v[32 * i + 14 * c];
            for (int k = 0; k < 13; k++) l[k] = (uint32_t)rnd() & F29_M;
            l[13] = (uint32_t)rnd() & 0x3FFu;  // < 2^387 < q
        }
}

template <typename F>
static float best_of(F launch, int reps) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e30f;
    for (int r = 0; r < reps; r++) {
        hipEventRecord(e0);
        launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    return best;
}

static uint64_t checksum(const uint32_t *d, uint64_t words) {
    std::vector<uint32_t> h(words);
    hipMemcpy(h.data(), d, words * 4, hipMemcpyDeviceToHost);
    uint64_t cs = 1469598103934665603ULL;
    for (uint32_t w : h) cs = (cs ^ w) * 1099511628211ULL;
    return cs;
}

int main(int argc, char **argv) {
    const uint64_t npts = 1 << 22;  // 512 MiB of 128-B entries: past the Infinity Cache, as the table
    const uint64_t threads = (uint64_t)256 * 4 * 3 * 64 * 4;  // 4 rounds of 3 waves per SIMD
    const int L = argc > 1 ? atoi(argv[1]) : 48;
    std::vector<uint32_t> h;
    fill(h, npts);
    uint32_t *dp, *dout;
    hipMalloc(&dp, h.size() * 4);
    hipMalloc(&dout, threads * 56 * 4);
    hipMemcpy(dp, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 2; rep++) {  // interleaved rounds (clock drift)
        for (int K = 0; K < 2; K++) {
            hipFuncAttributes fa;
            hipFuncGetAttributes(&fa, K ? (const void *)k_madd<true> : (const void *)k_madd<false>);
            auto go = [&] {
                if (K) k_madd<true><<<threads / 256, 256>>>(dp, npts, L, dout);
                else k_madd<false><<<threads / 256, 256>>>(dp, npts, L, dout);
            };
            go();
            hipDeviceSynchronize();
            float ms = best_of(go, 5);
            printf("%-10s madd: %8.3f ms  %.3f Gmadd/s  vgpr %3d  checksum %016llx\n",
                   K ? "karatsuba" : "schoolbook", ms, threads * (double)L / ms / 1e6, fa.numRegs,
                   (unsigned long long)checksum(dout, threads * 56));
        }
        for (int K = 0; K < 2; K++) {
            hipFuncAttributes fa;
            hipFuncGetAttributes(&fa, K ? (const void *)k_mul<true> : (const void *)k_mul<false>);
            auto go = [&] {
                if (K) k_mul<true><<<threads / 256, 256>>>(dp, 4 * L, dout);
                else k_mul<false><<<threads / 256, 256>>>(dp, 4 * L, dout);
            };
            go();
            hipDeviceSynchronize();
            float ms = best_of(go, 5);
            printf("%-10s mul : %8.3f ms  %.2f Gmul/s  vgpr %3d  checksum %016llx\n", K ? "karatsuba" : "schoolbook",
                   ms, threads * 16.0 * L / ms / 1e6, fa.numRegs, (unsigned long long)checksum(dout, threads * 56));
        }
    }
    return 0;
}
