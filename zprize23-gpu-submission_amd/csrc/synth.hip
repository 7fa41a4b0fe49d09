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

// Satisfying random arithmetic circuit (bench / tests; mirrors
// tests/pnp_testlib.py satisfying_witness).  Row i < n_gates:
//   q_l a + q_r b + q_o c + q_4 d + q_hl a^5 + q_hr b^5 + q_h4 d^5 + q_c (+PI) = 0,
// b_i = a_pi(i) with pi(i) = (A i + 1) mod n_gates (2-cycles (b,i) <-> (a,pi(i))),
// c solved from the gate, q_arith = 1; padding rows have q_arith = 0 and
// identity sigma.  sigma_j(w^i) = k_j w^target (k = 1, 7, 13, 17).
__global__ void k_synth_circuit_(const uint64_t *a, uint64_t *b, uint64_t *c, const uint64_t *d,
                                 const uint64_t *ql, const uint64_t *qr, const uint64_t *qo,
                                 const uint64_t *q4, const uint64_t *qc, const uint64_t *qhl,
                                 const uint64_t *qhr, const uint64_t *qh4, uint64_t *qarith,
                                 uint64_t *s0, uint64_t *s1, uint64_t *s2, uint64_t *s3, uint64_t n,
                                 uint64_t ng, uint64_t A, uint64_t pi_pos, Fr pi, Fr omega, Fr k1,
                                 Fr k2, Fr k3) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fr wi = pow_u64(omega, i);
    store_fr(s2, i, k2 * wi);
    store_fr(s3, i, k3 * wi);
    if (i >= ng) {
        store_fr(s0, i, wi);
        store_fr(s1, i, k1 * wi);
        store_fr(qarith, i, Fr::zero());
        return;
    }
    uint64_t pi_i = (uint64_t)(((unsigned __int128)A * i + 1) % ng);
    Fr ai = load_fr(a, i), bi = load_fr(a, pi_i), di = load_fr(d, i);
    store_fr(b, i, bi);
    store_fr(s1, i, pow_u64(omega, pi_i));
    store_fr(s0, pi_i, k1 * wi);
    auto p5 = [](const Fr &x) { Fr x2 = x * x; return x2 * x2 * x; };
    Fr acc = load_fr(ql, i) * ai + load_fr(qr, i) * bi + load_fr(q4, i) * di +
             load_fr(qhl, i) * p5(ai) + load_fr(qhr, i) * p5(bi) + load_fr(qh4, i) * p5(di) +
             load_fr(qc, i);
    if (i == pi_pos) acc = acc + pi;
    store_fr(c, i, neg(acc) * inverse(load_fr(qo, i)));
    store_fr(qarith, i, Fr::one());
}

void k_synth_circuit(uint64_t *const w[4], uint64_t *const sel[9], uint64_t *const sigma[4],
                     uint64_t n, uint64_t n_gates, uint64_t pi_pos, const Fr &pi_mont,
                     hipStream_t s) {
    uint64_t A = 0x9E3779B1ULL % n_gates;
    if (n_gates <= 2) A = 1;
    auto gcd = [](uint64_t x, uint64_t y) { while (y) { uint64_t t = x % y; x = y; y = t; } return x; };
    while (gcd(A, n_gates) != 1) A++;
    uint32_t lg = 0;
    while ((1ULL << lg) < n) lg++;
    const uint64_t root32[4] = {13381757501831005802ULL, 6564924994866501612ULL,
                                789602057691799140ULL, 6625830629041353339ULL};
    Fr omega = pow_u64(from_u64_limbs<FrP>(root32), 1ULL << (32 - lg));
    auto fr_small = [](uint32_t v) { Fr r = Fr::zero(); r.v[0] = v; return to_mont(r); };
    hipLaunchKernelGGL(k_synth_circuit_, dim3(nblk(n)), dim3(256), 0, s, w[0], w[1], w[2], w[3],
                       sel[0], sel[1], sel[2], sel[3], sel[4], sel[5], sel[6], sel[7], sel[8],
                       sigma[0], sigma[1], sigma[2], sigma[3], n, n_gates, A, pi_pos, pi_mont, omega,
                       fr_small(7), fr_small(13), fr_small(17));
    PNP_HIP(hipGetLastError());
}

}  // namespace pnp
