// FETCH_SIZE calibration for the accumulation's gather pattern (DESIGN §5,
// MI355X_MICROARCH.md HBM: "other access widths are uncalibrated"): every
// lane fetches one random 128-B table line as 7 x 16-B global_load_lds
// (112 B used), as k_accumulate29 does, over a 6 GiB table (far past the
// 256 MiB Infinity Cache).  Known bytes: lines x 128 (x 112 used).
//   rocprofv3 --pmc FETCH_SIZE -- ./ubench_gather
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glob_void_t;

__global__ __launch_bounds__(256) void k_gather(const uint32_t *table, uint64_t nlines, uint32_t steps,
                                                uint32_t *out) {
    __shared__ uint4 stage[4 * 7 * 64];
    const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    uint4 *wb = stage + 7 * 64 * wv;
    uint64_t x = (blockIdx.x * 256ULL + threadIdx.x) * 0x9E3779B97F4A7C15ULL + 1;
    uint32_t acc = 0;
    for (uint32_t s = 0; s < steps; s++) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        const uint32_t *p = table + 32 * (x % nlines);
#pragma unroll
        for (int c = 0; c < 7; c++)
            __builtin_amdgcn_global_load_lds((glob_void_t *)(p + 4 * c), (lds_void_t *)(wb + 64 * c), 16, 0, 0);
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
        const uint4 v = wb[ln];
        acc += v.x ^ v.w;
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main(int argc, char **argv) {
    // table size in GiB (argv[1], default 6): the folded SRS table is 6.5 GiB,
    // the copy-group table of HEIGHT = 15 35 GB (page-walk cost of random
    // gathers over it)
    const uint64_t gib = argc > 1 ? strtoull(argv[1], nullptr, 10) : 6;
    const uint64_t nlines = gib << 30 >> 7;
    uint32_t *table, *out;
    if (hipMalloc(&table, nlines * 128) != hipSuccess) return 1;
    hipMemset(table, 1, nlines * 128);
    const uint32_t blocks = 256 * 12, steps = 256;
    if (hipMalloc(&out, (size_t)blocks * 256 * 4) != hipSuccess) return 1;
    hipLaunchKernelGGL(k_gather, dim3(blocks), dim3(256), 0, 0, table, nlines, steps, out);  // warm
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_gather, dim3(blocks), dim3(256), 0, 0, table, nlines, steps, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double lines = (double)blocks * 256 * steps;
    printf("table %llu GiB: gathered lines per launch: %.0f  = %.3f GB at 128 B (%.3f GB used at 112 B); %.3f ms, %.1f GB/s (128 B)\n",
           (unsigned long long)gib, lines, lines * 128 / 1e9, lines * 112 / 1e9, ms, lines * 128 / (ms * 1e-3) / 1e9);
    return 0;
}
