// VGPR bank sensitivity of v_mad_u64_u32 on gfx950: 8 independent 64-bit
// accumulators, the two 32-bit sources in chosen registers (bank = index mod
// 4 on GCN/CDNA).  Prints cycles per wave64 instruction per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define ITERS 2048
#define R4(x) x x x x
#define MADS(S0, S1)                                                   \
    "v_mad_u64_u32 v[64:65], vcc, " S0 ", " S1 ", v[64:65]\n"          \
    "v_mad_u64_u32 v[66:67], vcc, " S0 ", " S1 ", v[66:67]\n"          \
    "v_mad_u64_u32 v[68:69], vcc, " S0 ", " S1 ", v[68:69]\n"          \
    "v_mad_u64_u32 v[70:71], vcc, " S0 ", " S1 ", v[70:71]\n"          \
    "v_mad_u64_u32 v[72:73], vcc, " S0 ", " S1 ", v[72:73]\n"          \
    "v_mad_u64_u32 v[74:75], vcc, " S0 ", " S1 ", v[74:75]\n"          \
    "v_mad_u64_u32 v[76:77], vcc, " S0 ", " S1 ", v[76:77]\n"          \
    "v_mad_u64_u32 v[78:79], vcc, " S0 ", " S1 ", v[78:79]\n"
#define KB(NAME, S0, S1)                                                                        \
    __global__ void NAME(uint64_t *out, uint32_t a) {                                           \
        asm volatile("v_mov_b32 v40, %0\nv_mov_b32 v41, %0\nv_mov_b32 v42, %0\nv_mov_b32 v44, %0\n" \
                     "v_mov_b32 v48, %0\n" ::"v"(a + threadIdx.x)                                \
                     : "v40", "v41", "v42", "v44", "v48");                                        \
        for (int i = 0; i < ITERS; i++)                                                         \
            asm volatile(R4(R4(MADS(S0, S1)))::: "vcc", "v64", "v65", "v66", "v67", "v68", "v69", \
                         "v70", "v71", "v72", "v73", "v74", "v75", "v76", "v77", "v78", "v79");   \
        uint32_t r;                                                                             \
        asm volatile("v_mov_b32 %0, v64" : "=v"(r));                                            \
        out[blockIdx.x * blockDim.x + threadIdx.x] = r;                                         \
    }
KB(k_b01, "v40", "v41")   // sources in banks 0, 1; acc pairs in banks 0,1 / 2,3
KB(k_b02, "v40", "v42")   // banks 0, 2
KB(k_b00, "v40", "v44")   // both bank 0
KB(k_b00s, "v40", "v40")  // the same register twice
int main() {
    uint64_t *out;
    hipMalloc(&out, 1 << 26);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct { const char *n; void (*k)(uint64_t *, uint32_t); } ks[] = {
        {"srcs banks 0,1", k_b01}, {"srcs banks 0,2", k_b02}, {"srcs bank 0,0", k_b00}, {"src same reg", k_b00s}};
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 8, threads = 256;  // 8 waves per SIMD
    for (auto &k : ks) {
        hipLaunchKernelGGL(k.k, dim3(blocks), dim3(threads), 0, 0, out, 3u);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k.k, dim3(blocks), dim3(threads), 0, 0, out, 3u);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double instr = (double)blocks * threads / 64 * ITERS * 128;  // wave instructions
        const double simd_cycles = ms * 1e-3 * 2.4e9 * cus * 4;
        printf("%-18s %.3f ms  %.2f cyc per wave64 mad per SIMD\n", k.n, ms, simd_cycles / instr);
    }
    return 0;
}
