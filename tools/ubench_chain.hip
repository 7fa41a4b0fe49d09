// Latency microbenchmark of dependent XYZZ additions (the bucket reduction's
// regime: few lanes, long chains).  Build per Montgomery variant / outlining:
//   hipcc -O3 --offload-arch=gfx950 -DPNP_MONT_VARIANT=v [-DPNP_FQ_OUTLINE] -I<csrc> ubench_chain.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include "field.cuh"
#include "ec.cuh"
using namespace pnp;

__global__ __launch_bounds__(256) void k_chain(const uint64_t *pts, int L, uint64_t *out) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    Xyzz a = load_xyzz(pts + 24 * (t % 1024)), b = load_xyzz(pts + 24 * ((t + 1) % 1024));
#pragma unroll 1
    for (int i = 0; i < L; i++) {
        a = add(a, b);
        b = add(b, a);
    }
    store_xyzz(out + 24 * t, a);
}

int main() {
    std::vector<uint64_t> h(24 * 1024);
    uint64_t s = 88172645463325252ULL;
    for (auto &w : h) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; w = s & 0x0fffffffffffffffULL; }
    uint64_t *dp, *dout;
    hipMalloc(&dp, h.size() * 8);
    hipMalloc(&dout, (1 << 20) * 24 * 8);
    hipMemcpy(dp, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    hipFuncAttributes fa;
    hipFuncGetAttributes(&fa, (const void *)k_chain);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const int L = 16;
    for (int threads : {4096, 32768, 262144, 1048576}) {
        k_chain<<<threads / 256, 256>>>(dp, 2, dout);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        k_chain<<<threads / 256, 256>>>(dp, L, dout);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("variant %d outline %d: %7d lanes: %8.3f ms, %6.2f us per dependent add, %7.3f Gadd/s, vgpr %d scratch %d\n",
               PNP_MONT_VARIANT,
#ifdef PNP_FQ_OUTLINE
               1,
#else
               0,
#endif
               threads, ms, ms * 1e3 / (2 * L), threads * 2.0 * L / ms / 1e6, fa.numRegs, (int)fa.localSizeBytes);
    }
    return 0;
}
