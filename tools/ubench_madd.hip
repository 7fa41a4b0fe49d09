// Microbenchmark of the MSM bucket loop: XYZZ mixed additions of randomly
// gathered affine points (as k_accumulate), per Montgomery-product variant
// (PNP_MONT_VARIANT, field.cuh).  Prints madd/s, VGPRs and a checksum that
// must agree across variants.
//   hipcc -O3 --offload-arch=gfx950 -DPNP_MONT_VARIANT=v -I<csrc> ubench_madd.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include "field.cuh"
#include "ec.cuh"
using namespace pnp;

__global__ __launch_bounds__(256) void k_bench(const uint64_t *pts, uint64_t npts, int L,
                                               uint64_t *out) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    Xyzz acc = Xyzz::inf();
    uint64_t h = t * 0x9E3779B97F4A7C15ULL;
    for (int i = 0; i < L; i++) {
        h = h * 6364136223846793005ULL + 1442695040888963407ULL;
        uint64_t idx = (h >> 20) % npts;
        const uint64_t *p = pts + 12 * idx;
        Fq x = load_fq(p), y = load_fq(p + 6);
        if (h & 1) y = neg(y);
        acc = madd(acc, x, y);
    }
    store_xyzz(out + 24 * t, acc);
}

__global__ void k_fq_chain(uint64_t *out, int L) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    Fq a = Fq::one(), b = Fq::one();
    a.v[0] += (uint32_t)t;
    b.v[1] += (uint32_t)t;
    Fq c = a, d = b;
    for (int i = 0; i < L; i++) {  // 4 independent products per iteration
        a = a * b; c = c * d; b = b * c; d = d * a;
    }
    store_fq(out + 6 * t, a + b + c + d);
}

int main() {
    const uint64_t npts = 1 << 22;
    const int L = 64;
    const uint64_t threads = 1 << 20;
    std::vector<uint64_t> h(12 * npts);
    uint64_t s = 88172645463325252ULL;
    for (auto &w : h) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; w = s; }
    for (uint64_t i = 0; i < npts; i++) { h[12 * i + 5] &= 0x0fffffffffffffffULL; h[12 * i + 11] &= 0x0fffffffffffffffULL; }
    uint64_t *dp, *dout;
    hipMalloc(&dp, h.size() * 8);
    hipMalloc(&dout, threads * 24 * 8);
    hipMemcpy(dp, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    hipFuncAttributes fa;
    hipFuncGetAttributes(&fa, (const void *)k_bench);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    k_bench<<<threads / 256, 256>>>(dp, npts, 4, dout);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 3; r++) {
        hipEventRecord(e0);
        k_bench<<<threads / 256, 256>>>(dp, npts, L, dout);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    std::vector<uint64_t> o(threads * 24);
    hipMemcpy(o.data(), dout, o.size() * 8, hipMemcpyDeviceToHost);
    uint64_t cs = 0;
    for (auto w : o) cs = cs * 1099511628211ULL + w;
    printf("variant %d: madd %.3f ms, %.3f Gmadd/s, vgpr %d, checksum %016llx\n", PNP_MONT_VARIANT,
           best, threads * (double)L / best / 1e6, fa.numRegs, (unsigned long long)cs);
    hipFuncGetAttributes(&fa, (const void *)k_fq_chain);
    best = 1e30f;
    for (int r = 0; r < 3; r++) {
        hipEventRecord(e0);
        k_fq_chain<<<threads / 256, 256>>>(dout, 256);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    hipMemcpy(o.data(), dout, threads * 6 * 8, hipMemcpyDeviceToHost);
    cs = 0;
    for (uint64_t i = 0; i < threads * 6; i++) cs = cs * 1099511628211ULL + o[i];
    printf("variant %d: fq_mul %.3f ms, %.2f Gmul/s, vgpr %d, checksum %016llx\n", PNP_MONT_VARIANT,
           best, threads * 256.0 * 4 / best / 1e6, fa.numRegs, (unsigned long long)cs);
    return 0;
}
