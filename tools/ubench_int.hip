// Microbenchmark: per-instruction VALU throughput on gfx950 (for the field
// multiplication design).  Each thread runs ITERS x 16 independent
// instructions of one kind; rate = lanes*instr / time.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 4096
#define REP16(x) x x x x x x x x x x x x x x x x

__global__ void k_mad64(uint64_t *out, uint32_t a, uint32_t b) {
    uint64_t acc0 = threadIdx.x, acc1 = acc0 + 1, acc2 = acc0 + 2, acc3 = acc0 + 3;
    uint32_t x = a + threadIdx.x, y = b;
    for (int i = 0; i < ITERS; i++) {
        asm volatile(REP16("v_mad_u64_u32 %0, vcc, %4, %5, %0\n v_mad_u64_u32 %1, vcc, %4, %5, %1\n v_mad_u64_u32 %2, vcc, %4, %5, %2\n v_mad_u64_u32 %3, vcc, %4, %5, %3\n")
                     : "+v"(acc0), "+v"(acc1), "+v"(acc2), "+v"(acc3) : "v"(x), "v"(y) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc0 + acc1 + acc2 + acc3;
}
__global__ void k_mullo(uint64_t *out, uint32_t a, uint32_t b) {
    uint32_t r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3;
    uint32_t x = a + threadIdx.x;
    for (int i = 0; i < ITERS; i++) {
        asm volatile(REP16("v_mul_lo_u32 %0, %0, %4\n v_mul_lo_u32 %1, %1, %4\n v_mul_lo_u32 %2, %2, %4\n v_mul_lo_u32 %3, %3, %4\n")
                     : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3) : "v"(x));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r0 + r1 + r2 + r3;
}
__global__ void k_mulhi(uint64_t *out, uint32_t a, uint32_t b) {
    uint32_t r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3;
    uint32_t x = a + threadIdx.x;
    for (int i = 0; i < ITERS; i++) {
        asm volatile(REP16("v_mul_hi_u32 %0, %0, %4\n v_mul_hi_u32 %1, %1, %4\n v_mul_hi_u32 %2, %2, %4\n v_mul_hi_u32 %3, %3, %4\n")
                     : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3) : "v"(x));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r0 + r1 + r2 + r3;
}
__global__ void k_addc(uint64_t *out, uint32_t a, uint32_t b) {
    uint32_t r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3;
    uint32_t x = a + threadIdx.x;
    for (int i = 0; i < ITERS; i++) {
        asm volatile(REP16("v_add_co_u32 %0, vcc, %0, %4\n v_addc_co_u32 %1, vcc, %1, %4, vcc\n v_addc_co_u32 %2, vcc, %2, %4, vcc\n v_addc_co_u32 %3, vcc, %3, %4, vcc\n")
                     : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3) : "v"(x) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r0 + r1 + r2 + r3;
}
__global__ void k_mov(uint64_t *out, uint32_t a, uint32_t b) {
    uint32_t r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3;
    uint32_t x = a + threadIdx.x;
    for (int i = 0; i < ITERS; i++) {
        asm volatile(REP16("v_mov_b32 %0, %4\n v_mov_b32 %1, %0\n v_mov_b32 %2, %1\n v_mov_b32 %3, %2\n")
                     : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3) : "v"(x));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r0 + r1 + r2 + r3;
}
__global__ void k_fma64(uint64_t *out, uint32_t a, uint32_t b) {
    double r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3;
    double x = a * 1e-9, y = b * 1e-9;
    for (int i = 0; i < ITERS; i++) {
        asm volatile(REP16("v_fma_f64 %0, %4, %5, %0\n v_fma_f64 %1, %4, %5, %1\n v_fma_f64 %2, %4, %5, %2\n v_fma_f64 %3, %4, %5, %3\n")
                     : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3) : "v"(x), "v"(y));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(r0 + r1 + r2 + r3);
}
__global__ void k_lshladd64(uint64_t *out, uint32_t a, uint32_t b) {
    uint64_t r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3;
    uint64_t x = a + threadIdx.x;
    for (int i = 0; i < ITERS; i++) {
        asm volatile(REP16("v_lshl_add_u64 %0, %4, 0, %0\n v_lshl_add_u64 %1, %4, 0, %1\n v_lshl_add_u64 %2, %4, 0, %2\n v_lshl_add_u64 %3, %4, 0, %3\n")
                     : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3) : "v"(x));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r0 + r1 + r2 + r3;
}
__global__ void k_mad24(uint64_t *out, uint32_t a, uint32_t b) {
    uint32_t r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3;
    uint32_t x = a + threadIdx.x, y = b;
    for (int i = 0; i < ITERS; i++) {
        asm volatile(REP16("v_mad_u32_u24 %0, %4, %5, %0\n v_mad_u32_u24 %1, %4, %5, %1\n v_mad_u32_u24 %2, %4, %5, %2\n v_mad_u32_u24 %3, %4, %5, %3\n")
                     : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3) : "v"(x), "v"(y));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r0 + r1 + r2 + r3;
}

typedef void (*kfn)(uint64_t *, uint32_t, uint32_t);
int main() {
    const int blocks = 256 * 8, threads = 256;
    uint64_t *out;
    hipMalloc(&out, (size_t)blocks * threads * 8);
    struct { const char *name; kfn f; } ks[] = {
        {"v_mad_u64_u32", k_mad64}, {"v_mul_lo_u32", k_mullo}, {"v_mul_hi_u32", k_mulhi},
        {"v_add_co/addc_co_u32", k_addc}, {"v_mov_b32", k_mov}, {"v_fma_f64", k_fma64},
        {"v_lshl_add_u64", k_lshladd64}, {"v_mad_u32_u24", k_mad24}};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (auto &k : ks) {
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 3, 5);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        for (int r = 0; r < 3; r++) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 3, 5);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        double instr = 3.0 * blocks * threads * (double)ITERS * 64;
        double rate = instr / (ms * 1e-3);
        // per CU per clock at 2.4 GHz nominal
        printf("%-22s %8.3f ms  %8.2f T lane-instr/s  %6.1f lane-instr/clk/CU\n", k.name, ms / 3, rate / 1e12,
               rate / 256 / 2.4e9);
    }
    return 0;
}
