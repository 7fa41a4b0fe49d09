// Per-instruction VALU issue cost on gfx950 (cycles per wave64 instruction per
// SIMD), for the limb-arithmetic design: 8 independent chains per lane so
// latency is hidden; rate reported as lane-instr/clk/CU at 2.4 GHz.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define ITERS 2048
#define R8(x) x x x x x x x x
#define K32(NAME, INSTR)                                                                    \
    __global__ void NAME(uint64_t *out, uint32_t a) {                                       \
        uint32_t r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4,      \
                 r5 = r0 + 5, r6 = r0 + 6, r7 = r0 + 7, x = a + threadIdx.x;                \
        for (int i = 0; i < ITERS; i++) {                                                   \
            asm volatile(R8(INSTR("%0") INSTR("%1") INSTR("%2") INSTR("%3") INSTR("%4")     \
                                INSTR("%5") INSTR("%6") INSTR("%7"))                        \
                         : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5),       \
                           "+v"(r6), "+v"(r7)                                               \
                         : "v"(x) : "vcc", "s20", "s21", "s22", "s23");                                     \
        }                                                                                   \
        out[blockIdx.x * blockDim.x + threadIdx.x] = r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7; \
    }
#define I_ADD(r) "v_add_u32 " r ", " r ", %8\n"
#define I_ADDCO(r) "v_add_co_u32 " r ", vcc, " r ", %8\n"
#define I_ADDC3(r) "v_addc_co_u32_e64 " r ", s[20:21], " r ", %8, s[22:23]\n"
#define I_ADD3(r) "v_add3_u32 " r ", " r ", %8, " r "\n"
#define I_AND(r) "v_and_b32 " r ", " r ", %8\n"
#define I_ALIGN(r) "v_alignbit_b32 " r ", " r ", %8, 29\n"
#define I_MULLO(r) "v_mul_lo_u32 " r ", " r ", %8\n"
#define I_MAD24(r) "v_mad_u32_u24 " r ", " r ", %8, " r "\n"
#define I_CND(r) "v_cndmask_b32 " r ", " r ", %8, vcc\n"
#define I_CND64(r) "v_cndmask_b32_e64 " r ", " r ", %8, s[20:21]\n"
#define I_SUBB(r) "v_subb_co_u32 " r ", vcc, " r ", %8, vcc\n"
K32(k_add, I_ADD)
K32(k_addco, I_ADDCO)
K32(k_addc3, I_ADDC3)
K32(k_add3, I_ADD3)
K32(k_and, I_AND)
K32(k_align, I_ALIGN)
K32(k_mullo, I_MULLO)
K32(k_mad24, I_MAD24)
K32(k_cnd, I_CND)
K32(k_cnd64, I_CND64)
K32(k_subb, I_SUBB)
// a cndmask stream as compiled field code uses it: VCC produced by a compare
// right before (the mask written, then read)
__global__ void k_cnd_cmp(uint64_t *out, uint32_t a) {
    uint32_t r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, x = a + threadIdx.x;
    for (int i = 0; i < ITERS; i++) {
#define I_CC(r) "v_cmp_gt_u32 vcc, " r ", %4\n v_cndmask_b32 " r ", " r ", %4, vcc\n"
        asm volatile(R8(I_CC("%0") I_CC("%1") I_CC("%2") I_CC("%3")) : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3)
                     : "v"(x) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = r0 + r1 + r2 + r3;
}

#define K64(NAME, INSTR)                                                                    \
    __global__ void NAME(uint64_t *out, uint32_t a) {                                       \
        uint64_t r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4,      \
                 r5 = r0 + 5, r6 = r0 + 6, r7 = r0 + 7;                                     \
        uint32_t x = a + threadIdx.x, y = a * 3;                                            \
        for (int i = 0; i < ITERS; i++) {                                                   \
            asm volatile(R8(INSTR("%0") INSTR("%1") INSTR("%2") INSTR("%3") INSTR("%4")     \
                                INSTR("%5") INSTR("%6") INSTR("%7"))                        \
                         : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5),       \
                           "+v"(r6), "+v"(r7)                                               \
                         : "v"(x), "v"(y) : "vcc", "s20", "s21", "s22", "s23");                             \
        }                                                                                   \
        out[blockIdx.x * blockDim.x + threadIdx.x] = r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7; \
    }
#define I_MAD64(r) "v_mad_u64_u32 " r ", s[20:21], %8, %9, " r "\n"
#define I_MAD64V(r) "v_mad_u64_u32 " r ", vcc, %8, %9, " r "\n"
#define I_SHR64(r) "v_lshrrev_b64 " r ", 29, " r "\n"
#define I_LADD64(r) "v_lshl_add_u64 " r ", " r ", 0, " r "\n"
K64(k_mad64, I_MAD64)
K64(k_mad64v, I_MAD64V)
K64(k_shr64, I_SHR64)
K64(k_ladd64, I_LADD64)

// FP64 FMA (the 52-bit-limb alternative to radix-2^29 products)
__global__ void k_fma64(uint64_t *out, uint32_t a) {
    double r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4, r5 = r0 + 5, r6 = r0 + 6,
           r7 = r0 + 7, x = 1.0000001 + a, y = 0.9999999;
    for (int i = 0; i < ITERS; i++) {
#define I_FMA64(r) "v_fma_f64 " r ", %8, %9, " r "\n"
        asm volatile(R8(I_FMA64("%0") I_FMA64("%1") I_FMA64("%2") I_FMA64("%3") I_FMA64("%4") I_FMA64("%5")
                            I_FMA64("%6") I_FMA64("%7"))
                     : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7)
                     : "v"(x), "v"(y));
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7);
}

// dependent chain latency: one chain per lane, 1 wave per SIMD
__global__ void k_lat_mad(uint64_t *out, uint32_t a) {
    uint64_t r = threadIdx.x;
    uint32_t x = a + threadIdx.x, y = a * 3;
    for (int i = 0; i < ITERS; i++)
        asm volatile(R8(R8("v_mad_u64_u32 %0, vcc, %1, %2, %0\n")) : "+v"(r) : "v"(x), "v"(y) : "vcc");
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_lat_madc(uint64_t *out, uint32_t a) {
    uint64_t r = threadIdx.x;
    uint32_t h = 0, x = a + threadIdx.x, y = a * 3;
    for (int i = 0; i < ITERS; i++)
        asm volatile(R8(R8("v_mad_u64_u32 %0, vcc, %2, %3, %0\nv_addc_co_u32 %1, vcc, 0, %1, vcc\n"))
                     : "+v"(r), "+v"(h) : "v"(x), "v"(y) : "vcc");
    out[blockIdx.x * blockDim.x + threadIdx.x] = r + h;
}

typedef void (*kfn)(uint64_t *, uint32_t);
int main() {
    uint64_t *out;
    hipMalloc(&out, (size_t)256 * 8 * 256 * 8);
    struct { const char *name; kfn f; double per_iter; } ks[] = {
        {"v_add_u32", k_add, 64}, {"v_add_co_u32(vcc)", k_addco, 64}, {"v_addc_co_u32_e64", k_addc3, 64},
        {"v_add3_u32", k_add3, 64}, {"v_and_b32", k_and, 64}, {"v_alignbit_b32", k_align, 64},
        {"v_mul_lo_u32", k_mullo, 64}, {"v_mad_u32_u24", k_mad24, 64}, {"v_cndmask_b32", k_cnd, 64}, {"v_cndmask_b32_e64(sgpr)", k_cnd64, 64},
        {"v_subb_co_u32(vcc)", k_subb, 64}, {"v_cmp+v_cndmask pair", k_cnd_cmp, 32},
        {"v_mad_u64_u32(sdst)", k_mad64, 64}, {"v_mad_u64_u32(vcc)", k_mad64v, 64},
        {"v_lshrrev_b64", k_shr64, 64}, {"v_lshl_add_u64", k_ladd64, 64}, {"v_fma_f64", k_fma64, 64}};
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const int blocks = 256 * 8, threads = 256;
    for (auto &k : ks) {
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 3);
        hipDeviceSynchronize();
        hipEventRecord(e0);
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, out, 3);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        double instr = (double)blocks * threads * ITERS * k.per_iter;
        double per_cu_clk = instr / (ms * 1e-3) / 256 / 2.4e9;
        printf("%-22s %7.3f ms %6.1f lane-instr/clk/CU  = %4.2f cyc per wave64 instr per SIMD\n", k.name, ms,
               per_cu_clk, 64.0 / (per_cu_clk / 4));
    }
    for (auto k : {std::make_pair("latency mad64 chain", k_lat_mad), std::make_pair("latency mad64+addc chain", k_lat_madc)}) {
        hipLaunchKernelGGL(k.second, dim3(256 * 4), dim3(64), 0, 0, out, 3);  // 1 wave per SIMD
        hipDeviceSynchronize();
        hipEventRecord(e0);
        hipLaunchKernelGGL(k.second, dim3(256 * 4), dim3(64), 0, 0, out, 3);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("%-26s %.1f cycles per link at 2.4 GHz\n", k.first, ms * 1e-3 * 2.4e9 / (ITERS * 64.0));
    }
    return 0;
}
