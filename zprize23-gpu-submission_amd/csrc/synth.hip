// synth.hip — synthetic-input generators for the bench / tests (not on the
// proving path): an SRS [tau^i] G and the 8n-coset constants that a real
// prover key carries (linear_evaluations = coset points, v_h_coset_8n).
#include "pnp_internal.h"
#include "ec.cuh"

namespace pnp {

static inline uint32_t nblk(uint64_t threads, uint32_t bs = 256) {
    return (uint32_t)((threads + bs - 1) / bs);
}

// canonical BLS12-381 G1 generator
static Fq g1_gen_x() {
    const uint64_t x[6] = {0xfb3af00adb22c6bbULL, 0x6c55e83ff97a1aefULL, 0xa14e3a3f171bac58ULL,
                           0xc3688c4f9774b905ULL, 0x2695638c4fa9ac0fULL, 0x17f1d3a73197d794ULL};
    return to_mont(from_u64_limbs<FqP>(x));
}
static Fq g1_gen_y() {
    const uint64_t y[6] = {0x0caa232946c5e7e1ULL, 0xd03cc744a2888ae4ULL, 0x00db18cb2c04b3edULL,
                           0xfcf5e095d5d00af6ULL, 0xa09e30ed741d8ae4ULL, 0x08b3f481e3aaa0f1ULL};
    return to_mont(from_u64_limbs<FqP>(y));
}

__global__ __launch_bounds__(256) void k_srs_(uint64_t *out, uint64_t n, Fr tau, Fq gx, Fq gy,
                                              uint32_t chunk) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t lo = t * chunk;
    if (lo >= n) return;
    uint64_t hi = lo + chunk < n ? lo + chunk : n;
    Fr tp = pow_u64(tau, lo);
    for (uint64_t i = lo; i < hi; i++) {
        Fr s = from_mont(tp);
        Xyzz acc = Xyzz::inf();
        for (int b = 255; b >= 0; b--) {
            acc = dbl(acc);
            if ((s.v[b >> 5] >> (b & 31)) & 1) acc = madd(acc, gx, gy);
        }
        Fq x, y;
        if (acc.is_inf()) {
            x = Fq::zero();
            y = Fq::one();
        } else {
            x = acc.x * inverse(acc.zz);
            y = acc.y * inverse(acc.zzz);
        }
        store_fq(out + 12 * i, x);
        store_fq(out + 12 * i + 6, y);
        tp = tp * tau;
    }
}

void k_srs(uint64_t *d, uint64_t n, const Fr &tau, hipStream_t s) {
    if (!n) return;
    const uint32_t chunk = 4;
    uint64_t threads = (n + chunk - 1) / chunk;
    hipLaunchKernelGGL(k_srs_, dim3(nblk(threads)), dim3(256), 0, s, d, n, tau, g1_gen_x(),
                       g1_gen_y(), chunk);
    PNP_HIP(hipGetLastError());
}

// x_i = g * w_8n^i ; vh_i = x_i^n - 1 = g^n * w_8^(i mod 8) - 1
__global__ void k_coset_consts_(uint64_t *vh, uint64_t *x, uint64_t N8, Fr g, Fr w8n,
                                const uint64_t *vh8, uint32_t chunk) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t lo = t * chunk;
    if (lo >= N8) return;
    uint64_t hi = lo + chunk < N8 ? lo + chunk : N8;
    Fr xi = g * pow_u64(w8n, lo);
    for (uint64_t i = lo; i < hi; i++) {
        if (x) store_fr(x, i, xi);
        if (vh) store_fr(vh, i, load_fr(vh8, i & 7));
        xi = xi * w8n;
    }
}

void k_coset_consts(uint64_t *vh, uint64_t *x, uint32_t lg_n, hipStream_t s) {
    const uint64_t root32[4] = {13381757501831005802ULL, 6564924994866501612ULL,
                                789602057691799140ULL, 6625830629041353339ULL};
    Fr r32 = from_u64_limbs<FrP>(root32);
    uint64_t n = 1ULL << lg_n, N8 = n << 3;
    Fr w8n = pow_u64(r32, 1ULL << (32 - (lg_n + 3)));
    Fr w8 = pow_u64(r32, 1ULL << (32 - 3));
    Fr seven = Fr::zero();
    seven.v[0] = 7;
    Fr g = to_mont(seven);
    Fr gn = pow_u64(g, n);
    uint64_t h[8 * 4];
    Fr p = gn;
    for (int k = 0; k < 8; k++) {
        to_u64_limbs(p - Fr::one(), h + 4 * k);
        p = p * w8;
    }
    DevBuf vh8(8 * 32);
    PNP_HIP(hipMemcpyAsync(vh8.p, h, sizeof h, hipMemcpyHostToDevice, s));
    const uint32_t chunk = 64;
    hipLaunchKernelGGL(k_coset_consts_, dim3(nblk((N8 + chunk - 1) / chunk)), dim3(256), 0, s, vh, x,
                       N8, g, w8n, vh8.u64(), chunk);
    PNP_HIP(hipGetLastError());
    PNP_HIP(hipStreamSynchronize(s));  // vh8 is freed on return
}

}  // namespace pnp
