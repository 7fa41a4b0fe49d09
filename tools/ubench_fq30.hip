// Microbenchmark: throughput of the Fq Montgomery product on the whole chip
// (random operands, every CU busy for ~0.1-0.5 s, so the clock the chip holds
// under that load is part of the result), radix 2^29 with one 64-bit column
// accumulator (field29.cuh, 392 v_mad_u64_u32) against 13 x 30-bit limbs
// with two accumulators (product / reduction columns each fit 64 bits; 338
// multiply-adds, more shifts and adds).  The accumulation of the MSM is
// limited by the power the chip may draw (DVFS), so products/s at the held
// clock is the figure of merit, not the issue-cycle count.
//   hipcc -O3 --offload-arch=gfx950 -I<csrc> ubench_fq30.hip -o ubench_fq30
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include "field29.cuh"
using namespace pnp;

namespace f30 {
constexpr uint32_t M = 0x3FFFFFFFu;
__device__ constexpr uint32_t Q[13] = {0x3fffaaabu, 0x27fbffffu, 0x153ffffbu, 0x2affffacu, 0x30f6241eu,
                                       0x34a83dau,  0x112bf673u, 0x12e13ce1u, 0x2cd76477u, 0x1ed90d2eu,
                                       0x29a4b1bau, 0x3a8e5ff9u, 0x1a0111u};
constexpr uint32_t QINV = 0x3ffcfffdu;  // -q^-1 mod 2^30
struct F30 {
    uint32_t l[13];
};
// a b 2^-390: product columns and reduction columns in separate 64-bit
// accumulators (13 products of < 2^60 each fit; together they would not)
__device__ __forceinline__ F30 mul(const F30 &a, const F30 &b) {
    uint32_t m[13];
    F30 r;
    uint64_t ap = 0, ar = 0;
#pragma unroll
    for (int k = 0; k < 25; k++) {
#pragma unroll
        for (int i = (k > 12 ? k - 12 : 0); i <= (k < 12 ? k : 12); i++) ap += (uint64_t)a.l[i] * b.l[k - i];
#pragma unroll
        for (int i = (k > 12 ? k - 12 : 0); i < (k < 13 ? k : 13); i++) ar += (uint64_t)m[i] * Q[k - i];
        uint32_t lo = ((uint32_t)ap & M) + ((uint32_t)ar & M);
        if (k < 13) {
            m[k] = (lo * QINV) & M;
            const uint64_t t = (uint64_t)m[k] * Q[0] + (lo & M);  // low 30 bits become 0
            lo = (uint32_t)(t >> 30) + (lo >> 30);
            // carry: (ap + ar + m q0) >> 30 = ap>>30 + ar>>30 + ((lo30 + m q0) >> 30)
            ap >>= 30;
            ar = (ar >> 30) + lo;
        } else {
            r.l[k - 13] = lo & M;
            ap >>= 30;
            ar = (ar >> 30) + (lo >> 30);
        }
    }
    r.l[12] = (uint32_t)(ap + ar);
    return r;
}
}  // namespace f30

__global__ __launch_bounds__(256) void k_mul29(uint32_t *out, int L, uint32_t seed) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    F29 a, b, c, d;
    uint32_t h = seed ^ (t * 0x9E3779B9u);
    for (int i = 0; i < 14; i++) {
        h = h * 1664525u + 1013904223u; a.l[i] = h & F29_M;
        h = h * 1664525u + 1013904223u; b.l[i] = h & F29_M;
        h = h * 1664525u + 1013904223u; c.l[i] = h & F29_M;
        h = h * 1664525u + 1013904223u; d.l[i] = h & F29_M;
    }
    a.l[13] &= 0xFFFFFF; b.l[13] &= 0xFFFFFF; c.l[13] &= 0xFFFFFF; d.l[13] &= 0xFFFFFF;
#pragma unroll 1
    for (int i = 0; i < L; i++) {
        a = mul29(a, b); c = mul29(c, d); b = mul29(b, c); d = mul29(d, a);
    }
    uint32_t x = 0;
    for (int i = 0; i < 14; i++) x ^= a.l[i] ^ b.l[i] ^ c.l[i] ^ d.l[i];
    out[t] = x;
}

__global__ __launch_bounds__(256) void k_mul30(uint32_t *out, int L, uint32_t seed) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    f30::F30 a, b, c, d;
    uint32_t h = seed ^ (t * 0x9E3779B9u);
    for (int i = 0; i < 13; i++) {
        h = h * 1664525u + 1013904223u; a.l[i] = h & f30::M;
        h = h * 1664525u + 1013904223u; b.l[i] = h & f30::M;
        h = h * 1664525u + 1013904223u; c.l[i] = h & f30::M;
        h = h * 1664525u + 1013904223u; d.l[i] = h & f30::M;
    }
    a.l[12] &= 0x3FFFFF; b.l[12] &= 0x3FFFFF; c.l[12] &= 0x3FFFFF; d.l[12] &= 0x3FFFFF;
#pragma unroll 1
    for (int i = 0; i < L; i++) {
        a = f30::mul(a, b); c = f30::mul(c, d); b = f30::mul(b, c); d = f30::mul(d, a);
    }
    uint32_t x = 0;
    for (int i = 0; i < 13; i++) x ^= a.l[i] ^ b.l[i] ^ c.l[i] ^ d.l[i];
    out[t] = x;
}

template <typename K>
static double run(K kern, const char *name, uint32_t *dout, uint32_t threads, int L) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(threads / 256), dim3(256), 0, 0, dout, 4, 1u);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(kern, dim3(threads / 256), dim3(256), 0, 0, dout, L, 7u + rep);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    hipFuncAttributes fa;
    hipFuncGetAttributes(&fa, (const void *)kern);
    const double prods = 4.0 * L * threads;
    printf("%-8s %8.3f ms  %7.2f G products/s  (%d VGPRs)\n", name, best, prods / best / 1e6, fa.numRegs);
    return prods / best / 1e6;
}

int main() {
    const uint32_t threads = 1u << 20;
    const int L = 256;
    uint32_t *dout;
    hipMalloc(&dout, threads * 4);
    double a = run(k_mul29, "mul29", dout, threads, L);
    double b = run(k_mul30, "mul30x2", dout, threads, L);
    a = run(k_mul29, "mul29", dout, threads, L);
    b = run(k_mul30, "mul30x2", dout, threads, L);
    printf("ratio mul30x2 / mul29 = %.3f\n", b / a);
    return 0;
}
