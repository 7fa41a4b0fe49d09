// Latency of dependent radix-2^29 XYZZ additions (the bucket reduction's
// regime: one wave per SIMD, long chains): xadd29 (products one after
// another) vs xadd29_ilp (independent products in interleaved pairs), and a
// bit-for-bit comparison of the two.
//   hipcc -O3 --offload-arch=gfx950 -I<csrc> ubench_chain29.hip -o ubench_chain29
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include "ec29.cuh"
using namespace pnp;

// Two independent Montgomery products a b and c d in one pass over the
// columns: the same column sums and digits as two mul29 calls (bit-identical
// results), with the two accumulator chains interleaved.
__device__ __forceinline__ void mul29x2(const F29 &a, const F29 &b, const F29 &c, const F29 &d, F29 &r, F29 &s) {
    uint32_t m[14], n[14];
    uint64_t acc = 0, acd = 0;
#pragma unroll
    for (int k = 0; k < 27; k++) {
#pragma unroll
        for (int i = (k > 13 ? k - 13 : 0); i <= (k < 13 ? k : 13); i++) {
            acc = mad29(a.l[i], b.l[k - i], acc);
            acd = mad29(c.l[i], d.l[k - i], acd);
        }
#pragma unroll
        for (int i = (k > 13 ? k - 13 : 0); i < (k < 14 ? k : 14); i++) {
            acc = mad29q(m[i], F29_Q[k - i], acc);
            acd = mad29q(n[i], F29_Q[k - i], acd);
        }
        if (k < 14) {
            m[k] = ((uint32_t)acc * F29_QINV) & F29_M;
            n[k] = ((uint32_t)acd * F29_QINV) & F29_M;
            acc = mad29q(m[k], F29_Q[0], acc);
            acd = mad29q(n[k], F29_Q[0], acd);
        } else {
            r.l[k - 14] = (uint32_t)acc & F29_M;
            s.l[k - 14] = (uint32_t)acd & F29_M;
        }
        acc >>= 29;
        acd >>= 29;
    }
    r.l[13] = (uint32_t)acc;
    s.l[13] = (uint32_t)acd;
}

// xadd29 with its independent products in pairs (mul29(R, R) = sqr29(R):
// the same column sums): ~5 product-times deep instead of ~12
__device__ __forceinline__ Xyzz29 xadd29_ilp(const Xyzz29 &p, const Xyzz29 &q) {
    F29 u1, t1, s1, t2, zz12, zzz12, pp, rr, ppp, qq;
    mul29x2(p.x, q.zz, q.x, p.zz, u1, t1);
    mul29x2(p.y, q.zzz, q.y, p.zzz, s1, t2);
    const F29 P = sub29(t1, u1, F29_KB), R = sub29(t2, s1, F29_KB);
    mul29x2(p.zz, q.zz, p.zzz, q.zzz, zz12, zzz12);
    mul29x2(P, P, R, R, pp, rr);
    mul29x2(P, pp, u1, pp, ppp, qq);
    Xyzz29 r;
    mul29x2(zz12, pp, zzz12, ppp, r.zz, r.zzz);
    r.x = sub29(sub29(sub29(rr, ppp, F29_KA), qq, F29_KA), qq, F29_KA);
    r.y = mul2_29(R, sub29(qq, r.x, F29_KB), s1, neg29(ppp, F29_KA));
    return r;
}

template <int V>
__global__ __launch_bounds__(256) void k_chain29(const uint32_t *pts, int L, uint32_t *out) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    Xyzz29 a = load_xyzz29(pts + 56 * (t % 1024)), b = load_xyzz29(pts + 56 * ((t + 1) % 1024));
#pragma unroll 1
    for (int i = 0; i < L; i++) {
        if (V == 0) {
            a = xadd29(a, b);
            b = xadd29(b, a);
        } else {
            a = xadd29_ilp(a, b);
            b = xadd29_ilp(b, a);
        }
    }
    store_xyzz29(out + 56 * t, a);
}

int main() {
    // inputs: random limbs < 2^29 for x, y; zz = zzz = small random (valid bounds
    // for the formulas; the values are not curve points — latency and the
    // equality of the two variants are what is measured)
    std::vector<uint32_t> h(56 * 1024);
    uint64_t s = 88172645463325252ULL;
    for (auto &w : h) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; w = (uint32_t)s & 0x1FFFFFFFu; }
    for (int p = 0; p < 1024; p++) { h[56 * p + 13] &= 0xF; h[56 * p + 27] &= 0xF; h[56 * p + 41] &= 0xF; h[56 * p + 55] &= 0xF; }
    const int threads = 256 * 256;  // one 256-lane block per CU: one wave per SIMD
    uint32_t *dp, *o0, *o1;
    hipMalloc(&dp, h.size() * 4);
    hipMalloc(&o0, (size_t)threads * 56 * 4);
    hipMalloc(&o1, (size_t)threads * 56 * 4);
    hipMemcpy(dp, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int L = 200;
    for (int v = 0; v < 2; v++) {
        for (int rep = 0; rep < 2; rep++) {
            hipEventRecord(e0);
            if (v == 0) hipLaunchKernelGGL(k_chain29<0>, dim3(threads / 256), dim3(256), 0, 0, dp, L, o0);
            else hipLaunchKernelGGL(k_chain29<1>, dim3(threads / 256), dim3(256), 0, 0, dp, L, o1);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep) printf("%s: %.2f us per dependent addition (one wave per SIMD)\n", v ? "xadd29_ilp" : "xadd29", 1e3 * ms / (2 * L));
        }
    }
    std::vector<uint32_t> a((size_t)threads * 56), b((size_t)threads * 56);
    hipMemcpy(a.data(), o0, a.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(b.data(), o1, b.size() * 4, hipMemcpyDeviceToHost);
    size_t diff = 0;
    for (size_t i = 0; i < a.size(); i++) diff += a[i] != b[i];
    printf("results %s (%zu differing words)\n", diff ? "DIFFER" : "identical", diff);
    return diff ? 1 : 0;
}
