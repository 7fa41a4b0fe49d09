// lagrange.hip — the commit key in the Lagrange basis of the size-n subgroup
// H = <omega>:
//     L_i = [L_i(tau)] G = (1/n) sum_j omega^(-i j) [tau^j] G,   i < n,
// i.e. the inverse NTT of the first n monomial SRS points, taken over G1.
//
// Why: the reference commits a witness polynomial from its coefficients
// (gen_proof.cuh:25-50: iNTT of the padded wire values, then the MSM over
// powers_of_g).  sum_j c_j [tau^j] G with c = iNTT(w) is the same group
// element as sum_i w_i L_i, so committing the evaluations over L gives the
// same commitment bytes — and an evaluation vector keeps the circuit's
// zeros: the rows past the last gate (1,032,380 of 2^22 for the HEIGHT = 15
// Merkle circuit, ~25%) and the zero-variable slots, whose digits drop out of
// the MSM's sort and accumulation.  The coefficients of the same polynomial
// are dense.
//
// Cost: one EC transform per (commit key, n), at the first commitment that
// needs it (like the folded table of the monomial key): log2(n) DIF layers of
// n/2 butterflies (a, b) -> (a + b, w^k (a - b)), one variable-base scalar
// multiplication per butterfly — GLV-split twiddle (two 128-bit halves),
// fixed 4-bit joint windows, the 15 multiples of the lane's point kept in a
// per-lane scratch table, so every lane of a wave runs the same 32 x (4
// doublings + 2 additions) whatever its twiddle (a bit-serial ladder would
// diverge on every bit).  1/n is folded into the first layer.  Point arithmetic: the radix-2^29
// XYZZ formulas of ec29.cuh for the scalar multiplications; the butterfly's
// sum and difference in exact 32-bit XYZZ (ec.cuh add: equal, opposite and
// infinite operands handled).  Outputs are bit-reversed by the DIF order and
// written back in natural order, affine (the commit-key format), ready for
// msm_build_table.
//
// Exceptional additions inside a scalar multiplication cannot occur (the
// accumulator holds (a + b lambda) P for prefixes a < lambda, b of the two
// halves, a + b lambda < r, never +- a window digit or its lambda multiple),
// so a zero ZZ at the end can only come from a degenerate key (a point of small
// order, tau a root of unity); it is flagged and the caller keeps committing
// from coefficients.
#include <algorithm>
#include "msm_internal.h"
#include "ec.cuh"
#include "ec29.cuh"

namespace pnp {

namespace {

constexpr int LAG_WIN = 4;                       // window bits
constexpr int LAG_TAB = (1 << LAG_WIN) - 1;      // multiples 1 .. 15 per lane
constexpr uint32_t LAG_PT = 56;                  // u32 per radix-2^29 XYZZ point

__global__ __launch_bounds__(256) void k_lag_load(const uint64_t *aff, uint64_t n, uint32_t *P) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    Xyzz p;
    p.x = load_fq(aff + 12 * i);
    p.y = load_fq(aff + 12 * i + 6);
    p.zz = Fq::one();
    p.zzz = Fq::one();
    store_xyzz29(P + LAG_PT * i, from32(p));
}

// tw[e] = w^e (Montgomery), e < m
__global__ __launch_bounds__(256) void k_lag_powers(uint64_t *tw, uint64_t m, Fr w) {
    const uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (e >= m) return;
    Fr acc = Fr::one(), b = w;
    for (uint64_t k = e; k; k >>= 1) {
        if (k & 1) acc = acc * b;
        b = b * b;
    }
    store_fr(tw, e, acc);
}

// GLV on BLS12-381 G1: phi(x, y) = (beta x, y) = [lambda] P, with
// lambda = z^2 - 1 (128 bits, lambda^2 + lambda + 1 = 0 mod r) and beta the
// matching cube root of unity in Fq (the other root gives [lambda^2] P; the
// pair was checked against the oracle's scalar multiplication, and the whole
// basis against the oracle's MSM in tests/test_gpu_lagrange.py).  beta is in
// the R = 2^406 form of field29.cuh.
__device__ constexpr uint32_t GLV_LAMBDA[4] = {0xffffffffu, 0x00000000u, 0x0001a402u, 0xac45a401u};
__device__ constexpr uint32_t GLV_BETA29[14] = {0x1195dfebu, 0x1b04e484u, 0x6026044u, 0x86070a2u, 0x1fd68858u,
                                                0x137e9670u, 0x6871e67u, 0x1e736664u, 0x83b24f6u, 0x8a70373u,
                                                0x2a012fdu, 0x112f94bu, 0x18a2733cu, 0x3u};

// s = s1 + s2 lambda, s1 < lambda, s2 = floor(s / lambda) < 2^128 (s < r < 2^255):
// binary long division of the 256-bit s by lambda
__device__ __forceinline__ void glv_split(const uint32_t s[8], uint32_t s1[4], uint32_t s2[4]) {
    uint32_t rem[5] = {0, 0, 0, 0, 0}, q[4] = {0, 0, 0, 0};
#pragma unroll 1
    for (int b = 255; b >= 0; b--) {
        const uint32_t bit = (s[b >> 5] >> (b & 31)) & 1u;
#pragma unroll
        for (int i = 4; i > 0; i--) rem[i] = (rem[i] << 1) | (rem[i - 1] >> 31);
        rem[0] = (rem[0] << 1) | bit;
        uint32_t t[5], br = 0;
#pragma unroll
        for (int i = 0; i < 5; i++) {
            const uint64_t d = (uint64_t)rem[i] - (i < 4 ? GLV_LAMBDA[i] : 0u) - br;
            t[i] = (uint32_t)d;
            br = (uint32_t)(d >> 63);
        }
        if (!br) {
#pragma unroll
            for (int i = 0; i < 5; i++) rem[i] = t[i];
            if (b < 128) q[b >> 5] |= 1u << (b & 31);  // the quotient is < 2^128
        }
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        s1[i] = rem[i];
        s2[i] = q[i];
    }
}

// s P for a canonical scalar s (8 x 32-bit limbs, s < r), P not infinity;
// tab: this lane's 15-point scratch table (j P, j = 1..15).  GLV: s = s1 +
// s2 lambda, both < 2^128, so 32 joint windows of 4 bits: 4 doublings, then
// s1's digit times P and s2's digit times phi(P) (the table entry with X times
// beta) — ~2.4k instead of ~3.4k Fq products per multiplication.  *bad set
// when the result is degenerate (ZZ = 0 mod q).
__device__ __forceinline__ Xyzz29 lag_smul(const Xyzz29 &P, const uint32_t *s, uint32_t *tab, uint32_t *bad) {
    {
        Xyzz29 T = P;
        store_xyzz29(tab, T);
        T = xdbl29(P);
        store_xyzz29(tab + LAG_PT, T);
#pragma unroll 1
        for (int k = 3; k <= LAG_TAB; k++) {
            T = xadd29(T, P);
            store_xyzz29(tab + LAG_PT * (k - 1), T);
        }
    }
    uint32_t s1[4], s2[4];
    glv_split(s, s1, s2);
    Xyzz29 acc = P;
    bool started = false;
#pragma unroll 1
    for (int w = 128 / LAG_WIN - 1; w >= 0; w--) {
        if (started) {
#pragma unroll 1
            for (int d = 0; d < LAG_WIN; d++) acc = xdbl29(acc);
        }
        const int bit = w * LAG_WIN;
#pragma unroll 1
        for (int j = 0; j < 2; j++) {  // one addition site: s1's digit, then s2's
            const uint32_t dig = ((j ? s2 : s1)[bit >> 5] >> (bit & 31)) & LAG_TAB;
            if (dig) {
                Xyzz29 Q = load_xyzz29(tab + LAG_PT * (dig - 1));
                if (j) Q.x = mul29(Q.x, const29(GLV_BETA29));
                acc = started ? xadd29(acc, Q) : Q;
                started = true;
            }
        }
    }
    if (!started || zero29(acc.zz)) *bad = 1u;
    return acc;
}

__device__ __forceinline__ void canon_limbs(const Fr &a_mont, uint32_t s[8]) {
    const Fr c = from_mont(a_mont);
#pragma unroll
    for (int i = 0; i < 8; i++) s[i] = c.v[i];
}

// one DIF layer of half-size h over the n points P (radix 2^29 XYZZ):
// (a, b) -> (a + b, w^k (a - b)), w^k = tw[k * stride]; scale != 1: both
// outputs also times scale (the first layer carries the 1/n)
__global__ __launch_bounds__(256) void k_lag_layer(uint32_t *P, uint64_t n, uint64_t h, const uint64_t *tw,
                                                   uint64_t stride, Fr scale, int scaled, uint32_t *scratch,
                                                   uint64_t lanes, uint32_t *bad) {
    const uint64_t lane = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (lane >= lanes) return;
    uint32_t *tab = scratch + (uint64_t)LAG_TAB * LAG_PT * lane;
#pragma unroll 1
    for (uint64_t j = lane; j < n / 2; j += lanes) {
        const uint64_t blk = j / h, k = j - blk * h;
        const uint64_t i0 = 2 * h * blk + k, i1 = i0 + h;
        const Xyzz a = to32(load_xyzz29(P + LAG_PT * i0)), b = to32(load_xyzz29(P + LAG_PT * i1));
        Xyzz nb = b;
        nb.y = Fq::zero() - b.y;
        const Xyzz sum = add(a, b), dif = add(a, nb);
        // one scalar multiplication site (inlined once): job 0 = the sum
        // (first layer only: times 1/n), job 1 = the difference times w^k
#pragma unroll 1
        for (int job = 0; job < 2; job++) {
            const uint64_t dst = job ? i1 : i0;
            const Xyzz &pt = job ? dif : sum;
            if (job == 0 ? !scaled : (k == 0 && !scaled)) {
                store_xyzz29(P + LAG_PT * dst, from32(pt));
                continue;
            }
            uint32_t sc[8];
            canon_limbs(job ? load_fr(tw, k * stride) * scale : scale, sc);
            store_xyzz29(P + LAG_PT * dst, pt.is_inf() ? inf29() : lag_smul(from32(pt), sc, tab, bad));
        }
    }
}

// natural order out of the bit-reversed DIF output, 32-bit XYZZ (24 u64)
__global__ __launch_bounds__(256) void k_lag_out(const uint32_t *P, uint64_t n, int lg, uint64_t *xyzz,
                                                 uint32_t *bad) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t r = lg ? (__brevll(i) >> (64 - lg)) : 0;
    const Xyzz p = to32(load_xyzz29(P + LAG_PT * r));
    if (p.is_inf()) *bad = 1u;  // L_i(tau) = 0: tau in H
    store_xyzz(xyzz + 24 * i, p);
}

}  // namespace

bool srs_lagrange(const uint64_t *d_aff, uint64_t n, const Fr &omega_inv, const Fr &n_inv, uint64_t *d_out,
                  hipStream_t s) {
    if (n < 2 || (n & (n - 1))) return false;
    int lg = 0;
    while ((1ULL << lg) < n) lg++;
    DevBuf P(n * LAG_PT * 4), tw((n / 2) * 32), flag(16);
    uint32_t *bad = static_cast<uint32_t *>(flag.p);
    PNP_HIP(hipMemsetAsync(bad, 0, 4, s));
    hipLaunchKernelGGL(k_lag_load, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, d_aff, n,
                       static_cast<uint32_t *>(P.p));
    PNP_HIP(hipGetLastError());
    bg_step(s);
    hipLaunchKernelGGL(k_lag_powers, dim3((uint32_t)((n / 2 + 255) / 256)), dim3(256), 0, s, tw.u64(), n / 2,
                       omega_inv);
    PNP_HIP(hipGetLastError());
    bg_step(s);
    // lanes: the whole layer when it fits 2^18 lanes (880 MB of window tables)
    const uint64_t lanes = std::min<uint64_t>(n / 2, 1ULL << 18);
    DevBuf scratch(lanes * LAG_TAB * LAG_PT * 4);
    for (uint64_t h = n / 2; h >= 1; h /= 2) {
        const bool first = h == n / 2;
        hipLaunchKernelGGL(k_lag_layer, dim3((uint32_t)((lanes + 255) / 256)), dim3(256), 0, s,
                           static_cast<uint32_t *>(P.p), n, h, tw.u64(), (n / 2) / h, first ? n_inv : Fr::one(),
                           (int)first, static_cast<uint32_t *>(scratch.p), lanes, bad);
        PNP_HIP(hipGetLastError());
        bg_step(s);
    }
    DevBuf X(n * 192);
    hipLaunchKernelGGL(k_lag_out, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s,
                       static_cast<const uint32_t *>(P.p), n, lg, X.u64(), bad);
    PNP_HIP(hipGetLastError());
    bg_step(s);
    xyzz_to_affine_dev(X.u64(), n, d_out, s);
    uint32_t hbad = 0;
    PNP_HIP(hipMemcpyAsync(&hbad, bad, 4, hipMemcpyDeviceToHost, s));
    PNP_HIP(hipStreamSynchronize(s));
    return hbad == 0;
}

}  // namespace pnp
