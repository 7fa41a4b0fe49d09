// poly.hip — generic Fr vector kernels used along the gen_proof path.
//
// Reference operators restated (utils/mont/cuda/mont_arithmetic.cu):
//   accumulate_mul_poly :334-360  exclusive prefix product (z, z2 grand products)
//   poly_div_cuda       :305-331  quotient by (X - z), remainder dropped
//   evaluate            :105-173  sum c_i x^i (function.cu:162-173)
//   inv_mod             :73       per-element inverse (inv(0) = 0)
// The reference runs log2(N) Hillis-Steele passes over the whole array (22 at
// N = 2^22) and a per-thread square-and-multiply for x^i.  Here every scan is
// a chunked recursion: each lane folds a chunk of K consecutive elements,
// the chunk totals recurse (N -> N/K -> ...), then each lane re-walks its
// chunk with its carry.  Work is ~2-3 multiplications per element and a
// handful of launches, with every global access coalesced per chunk row.
#include "pnp_internal.h"

namespace pnp {

static constexpr int CHUNK = 32;

static inline uint32_t nblk(uint64_t threads, uint32_t bs = 256) {
    return (uint32_t)((threads + bs - 1) / bs);
}

// ---------------------------------------------------------------- conversions
__global__ void k_from_mont_(uint64_t *d, uint64_t n) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < n) store_fr(d, i, from_mont(load_fr(d, i)));
}
__global__ void k_to_mont_(uint64_t *d, uint64_t n) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < n) store_fr(d, i, to_mont(load_fr(d, i)));
}
void k_from_mont(uint64_t *d, uint64_t n, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_from_mont_, dim3(nblk(n)), dim3(256), 0, s, d, n);
    PNP_HIP(hipGetLastError());
}
void k_to_mont(uint64_t *d, uint64_t n, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_to_mont_, dim3(nblk(n)), dim3(256), 0, s, d, n);
    PNP_HIP(hipGetLastError());
}

// ---------------------------------------------------------------- prefix product
// chunk c = [cK, cK+K): tot[c] = prod of the chunk
__global__ void k_chunk_prod(const uint64_t *d, uint64_t n, uint64_t *tot) {
    uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t lo = c * CHUNK;
    if (lo >= n) return;
    uint64_t hi = lo + CHUNK < n ? lo + CHUNK : n;
    Fr acc = load_fr(d, lo);
    for (uint64_t i = lo + 1; i < hi; i++) acc = acc * load_fr(d, i);
    store_fr(tot, c, acc);
}
// d[i] <- carry * prod_{chunk start <= j < i} d[j]; carry = exclusive prefix of chunk totals
__global__ void k_chunk_prod_apply(uint64_t *d, uint64_t n, const uint64_t *pre) {
    uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t lo = c * CHUNK;
    if (lo >= n) return;
    uint64_t hi = lo + CHUNK < n ? lo + CHUNK : n;
    Fr acc = load_fr(pre, c);
    for (uint64_t i = lo; i < hi; i++) {
        Fr x = load_fr(d, i);
        store_fr(d, i, acc);
        acc = acc * x;
    }
}
__global__ void k_seq_prefix_prod(uint64_t *d, uint64_t n) {
    Fr acc = Fr::one();
    for (uint64_t i = 0; i < n; i++) {
        Fr x = load_fr(d, i);
        store_fr(d, i, acc);
        acc = acc * x;
    }
}
static void prefix_product_rec(uint64_t *d, uint64_t n, uint64_t *scratch, hipStream_t s) {
    if (n <= CHUNK) {
        hipLaunchKernelGGL(k_seq_prefix_prod, dim3(1), dim3(1), 0, s, d, n);
        PNP_HIP(hipGetLastError());
        return;
    }
    uint64_t nc = (n + CHUNK - 1) / CHUNK;
    uint64_t *tot = scratch;
    hipLaunchKernelGGL(k_chunk_prod, dim3(nblk(nc)), dim3(256), 0, s, d, n, tot);
    PNP_HIP(hipGetLastError());
    prefix_product_rec(tot, nc, scratch + 4 * nc, s);
    hipLaunchKernelGGL(k_chunk_prod_apply, dim3(nblk(nc)), dim3(256), 0, s, d, n, tot);
    PNP_HIP(hipGetLastError());
}
static uint64_t rec_scratch_elems(uint64_t n) {
    uint64_t t = 0;
    while (n > CHUNK) { n = (n + CHUNK - 1) / CHUNK; t += n; }
    return t + 1;
}
void k_prefix_product(uint64_t *d, uint64_t n, DevBuf &scratch, hipStream_t s) {
    if (!n) return;
    size_t need = rec_scratch_elems(n) * 32;
    if (scratch.bytes < need) scratch.alloc(need);
    prefix_product_rec(d, n, scratch.u64(), s);
}

// ---------------------------------------------------------------- batch inverse
// Chunk c of nc holds the elements c, c + nc, c + 2 nc, ... (any partition
// serves a batch inverse): a wave's loads and stores are 64 consecutive
// elements, not 64 elements a chunk (1 KB) apart as with contiguous chunks.
__global__ void k_binv_up(const uint64_t *d, uint64_t n, uint64_t nc, uint64_t *pre, uint64_t *tot) {
    uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (c >= nc) return;
    Fr acc = Fr::one();
    for (uint64_t i = c; i < n; i += nc) {
        store_fr(pre, i, acc);
        Fr x = load_fr(d, i);
        if (!x.is_zero()) acc = acc * x;
    }
    store_fr(tot, c, acc);
}
__global__ void k_binv_down(uint64_t *d, uint64_t n, uint64_t nc, const uint64_t *pre, const uint64_t *tinv) {
    uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (c >= nc || c >= n) return;
    Fr acc = load_fr(tinv, c);
    for (uint64_t i = c + (n - 1 - c) / nc * nc;; i -= nc) {
        Fr x = load_fr(d, i);
        if (!x.is_zero()) {
            store_fr(d, i, acc * load_fr(pre, i));
            acc = acc * x;
        }
        if (i < nc) break;
    }
}
// The batch inverse's base case: <= 4096 independent inversions, one per
// lane, so its time is ONE inversion's latency: field.cuh fr_inverse_bin
// (binary extended Euclid) instead of Fermat's ~380 dependent products
// (0.3 ms, exposed at 8 ranks).
__global__ void k_inv_small(uint64_t *d, uint64_t n) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < n) store_fr(d, i, fr_inverse_bin(load_fr(d, i)));
}
static void binv_rec(uint64_t *d, uint64_t n, uint64_t *scratch, hipStream_t s) {
    if (n <= 4096) {
        hipLaunchKernelGGL(k_inv_small, dim3(nblk(n, 64)), dim3(64), 0, s, d, n);
        PNP_HIP(hipGetLastError());
        return;
    }
    uint64_t nc = (n + CHUNK - 1) / CHUNK;
    uint64_t *pre = scratch, *tot = scratch + 4 * n;
    hipLaunchKernelGGL(k_binv_up, dim3(nblk(nc)), dim3(256), 0, s, d, n, nc, pre, tot);
    PNP_HIP(hipGetLastError());
    binv_rec(tot, nc, tot + 4 * nc, s);
    hipLaunchKernelGGL(k_binv_down, dim3(nblk(nc)), dim3(256), 0, s, d, n, nc, pre, tot);
    PNP_HIP(hipGetLastError());
}
void k_batch_inverse(uint64_t *d, uint64_t n, DevBuf &scratch, hipStream_t s) {
    if (!n) return;
    uint64_t need = 0, m = n;
    while (m > 4096) { uint64_t nc = (m + CHUNK - 1) / CHUNK; need += m + nc; m = nc; }
    need = (need + 1) * 32;
    if (scratch.bytes < need) scratch.alloc(need);
    binv_rec(d, n, scratch.u64(), s);
}

// ---------------------------------------------------------------- suffix Horner
// H[k] = sum_{j >= k} v_j z^(j-k).  Chunk value L_c = H restricted to the chunk.
// Up to HB_MAX independent polys (each its own z) share every launch
// (blockIdx.y): the levels above the first are latency-bound chains of CHUNK
// dependent products, so the round-6 pair of divisions costs one chain, not two.
constexpr int HB_MAX = 4;
struct HornerSet {
    uint64_t *v[HB_MAX];
    Fr z[HB_MAX];
};
__global__ void k_horner_chunk(HornerSet hs, uint64_t n, uint64_t *L, uint64_t nc) {
    uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t lo = c * CHUNK;
    if (lo >= n) return;
    const uint64_t *v = hs.v[blockIdx.y];
    const Fr z = hs.z[blockIdx.y];
    uint64_t hi = lo + CHUNK < n ? lo + CHUNK : n;
    // two steps at a time, acc z^2 + v_(i+1) z + v_i: one reduction (fr_mul2)
    const Fr z2 = z * z;
    uint64_t i = hi;
    Fr acc = Fr::zero();
    if ((hi - lo) & 1) acc = load_fr(v, --i);
    while (i > lo) {
        i -= 2;
        acc = fr_mul2(acc, z2, load_fr(v, i + 1), z) + load_fr(v, i);
    }
    store_fr(L + 4 * nc * blockIdx.y, c, acc);
}
// H at chunk starts is in Hc (inclusive); write H[k] for every k of the chunk
// (mode 0) or the shifted quotient q[k] = H[k+1] (mode 1: poly division)
__global__ void k_horner_apply(HornerSet hs, uint64_t n, const uint64_t *Hc, uint64_t nc, int shift) {
    uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t lo = c * CHUNK;
    if (lo >= n) return;
    uint64_t *v = hs.v[blockIdx.y];
    const Fr z = hs.z[blockIdx.y];
    Hc += 4 * nc * blockIdx.y;
    uint64_t hi = lo + CHUNK < n ? lo + CHUNK : n;
    Fr acc = c + 1 < nc ? load_fr(Hc, c + 1) : Fr::zero();  // H[hi]
    for (uint64_t i = hi; i-- > lo;) {
        Fr x = load_fr(v, i);
        if (shift) store_fr(v, i, acc);
        acc = acc * z + x;
        if (!shift) store_fr(v, i, acc);
    }
}
__global__ void k_seq_horner(HornerSet hs, uint64_t n, int shift) {
    uint64_t *v = hs.v[blockIdx.y];
    const Fr z = hs.z[blockIdx.y];
    Fr acc = Fr::zero();
    for (uint64_t i = n; i-- > 0;) {
        Fr x = load_fr(v, i);
        if (shift) store_fr(v, i, acc);
        acc = acc * z + x;
        if (!shift) store_fr(v, i, acc);
    }
}
static void horner_rec(const HornerSet &hs, int K, uint64_t n, int shift, uint64_t *scratch, hipStream_t s) {
    if (n <= CHUNK) {
        hipLaunchKernelGGL(k_seq_horner, dim3(1, K), dim3(1), 0, s, hs, n, shift);
        PNP_HIP(hipGetLastError());
        return;
    }
    uint64_t nc = (n + CHUNK - 1) / CHUNK;
    uint64_t *L = scratch;  // K x nc
    hipLaunchKernelGGL(k_horner_chunk, dim3(nblk(nc), K), dim3(256), 0, s, hs, n, L, nc);
    PNP_HIP(hipGetLastError());
    HornerSet up = {};
    for (int k = 0; k < K; k++) {
        up.v[k] = L + 4 * nc * k;
        up.z[k] = pow_u64(hs.z[k], CHUNK);
    }
    horner_rec(up, K, nc, 0, scratch + 4 * nc * K, s);  // L <- inclusive H at chunk starts
    hipLaunchKernelGGL(k_horner_apply, dim3(nblk(nc), K), dim3(256), 0, s, hs, n, L, nc, shift);
    PNP_HIP(hipGetLastError());
}
void k_poly_div_linear_batch(uint64_t *const *d, const Fr *z, int K, uint64_t n, DevBuf &scratch,
                             hipStream_t s) {
    if (!n) return;
    for (int k0 = 0; k0 < K; k0 += HB_MAX) {
        const int kb = std::min(K - k0, HB_MAX);
        size_t need = rec_scratch_elems(n) * 32 * kb;
        if (scratch.bytes < need) scratch.alloc(need);
        HornerSet hs = {};
        for (int k = 0; k < kb; k++) {
            hs.v[k] = d[k0 + k];
            hs.z[k] = z[k0 + k];
        }
        horner_rec(hs, kb, n, 1, scratch.u64(), s);
    }
}
void k_poly_div_linear(uint64_t *d, uint64_t n, const Fr &z, DevBuf &scratch, hipStream_t s) {
    k_poly_div_linear_batch(&d, &z, 1, n, scratch, s);
}

// ---------------------------------------------------------------- evaluation
// partial[p][b] = sum over block b's 256 * EV_K coefficients of c_i x^i for
// each of NP polys.  Lane t of block b takes the coefficients
// base + t + 256 k (k < EV_K, coalesced loads), Horner in X = x^256, then one
// product by x^(base + t) = (x^(256 EV_K))^b x^t: a 9- and an 8-bit power per
// lane instead of the full x^lo power per 32-coefficient chunk of the
// previous layout (which cost more products than the Horner steps).
// 32 coefficients a lane: 16 (4 waves a SIMD at 2^22 instead of 2) measured
// slower, 1.06 vs 0.91 ms per proof: the lane's two powers (~25 products)
// are spread over half the coefficients (profiles/r05_ab_mul2_lincomb_eval.txt)
static constexpr int EV_K = 32;
struct EvalPtrs {  // up to 8 polys, by value in the kernel arguments (no upload)
    const uint64_t *p[8];
};
// Two Horner steps at a time, h <- h X^2 + c_k X + c_(k-1) (X = x^256): the
// two products share one Montgomery reduction (fr_mul2).
template <int NP>
__global__ __launch_bounds__(256) void k_eval_partial(EvalPtrs polys, uint64_t n, Fr x,
                                                      Fr x256, Fr xblk, uint64_t *partial) {
    static_assert(EV_K % 2 == 0, "Horner steps in pairs");
    __shared__ uint4 red_lo[256], red_hi[256];
    const uint64_t base = (uint64_t)blockIdx.x * 256 * EV_K + threadIdx.x;
    const Fr x512 = x256 * x256;
    Fr h[NP];
#pragma unroll
    for (int p = 0; p < NP; p++) h[p] = Fr::zero();
#pragma unroll 1
    for (int k = EV_K - 1; k >= 1; k -= 2) {
        const uint64_t i1 = base + 256ull * k, i0 = i1 - 256;  // i0 < i1
#pragma unroll
        for (int p = 0; p < NP; p++) {
            const Fr c1 = i1 < n ? load_fr(polys.p[p], i1) : Fr::zero();
            const Fr c0 = i0 < n ? load_fr(polys.p[p], i0) : Fr::zero();
            h[p] = fr_mul2(h[p], x512, c1, x256) + c0;
        }
    }
    const Fr sc = pow_u64(xblk, blockIdx.x) * pow_u64(x, threadIdx.x);  // x^(base)
#pragma unroll
    for (int p = 0; p < NP; p++) h[p] = h[p] * sc;
#pragma unroll
    for (int p = 0; p < NP; p++) {
        red_lo[threadIdx.x] = make_uint4(h[p].v[0], h[p].v[1], h[p].v[2], h[p].v[3]);
        red_hi[threadIdx.x] = make_uint4(h[p].v[4], h[p].v[5], h[p].v[6], h[p].v[7]);
        __syncthreads();
        for (int st = 128; st > 0; st >>= 1) {
            if ((int)threadIdx.x < st) {
                uint4 a0 = red_lo[threadIdx.x], a1 = red_hi[threadIdx.x];
                uint4 b0 = red_lo[threadIdx.x + st], b1 = red_hi[threadIdx.x + st];
                Fr a, b;
                a.v[0] = a0.x; a.v[1] = a0.y; a.v[2] = a0.z; a.v[3] = a0.w;
                a.v[4] = a1.x; a.v[5] = a1.y; a.v[6] = a1.z; a.v[7] = a1.w;
                b.v[0] = b0.x; b.v[1] = b0.y; b.v[2] = b0.z; b.v[3] = b0.w;
                b.v[4] = b1.x; b.v[5] = b1.y; b.v[6] = b1.z; b.v[7] = b1.w;
                Fr r = a + b;
                red_lo[threadIdx.x] = make_uint4(r.v[0], r.v[1], r.v[2], r.v[3]);
                red_hi[threadIdx.x] = make_uint4(r.v[4], r.v[5], r.v[6], r.v[7]);
            }
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            uint4 *dst = reinterpret_cast<uint4 *>(partial + 4 * ((uint64_t)p * gridDim.x + blockIdx.x));
            dst[0] = red_lo[0];
            dst[1] = red_hi[0];
        }
        __syncthreads();
    }
}
// sum partials per poly (single block per poly)
__global__ __launch_bounds__(256) void k_sum_partials(const uint64_t *partial, uint64_t nb,
                                                      uint64_t *out) {
    __shared__ uint4 red_lo[256], red_hi[256];
    const uint64_t *pp = partial + 4 * (uint64_t)blockIdx.x * nb;
    Fr acc = Fr::zero();
    for (uint64_t i = threadIdx.x; i < nb; i += 256) acc = acc + load_fr(pp, i);
    // a tree over the 256 lane sums (8 dependent additions, not 256 on one lane)
    for (int st = 128; st > 0; st >>= 1) {
        red_lo[threadIdx.x] = make_uint4(acc.v[0], acc.v[1], acc.v[2], acc.v[3]);
        red_hi[threadIdx.x] = make_uint4(acc.v[4], acc.v[5], acc.v[6], acc.v[7]);
        __syncthreads();
        if ((int)threadIdx.x < st) {
            Fr b;
            const uint4 b0 = red_lo[threadIdx.x + st], b1 = red_hi[threadIdx.x + st];
            b.v[0] = b0.x; b.v[1] = b0.y; b.v[2] = b0.z; b.v[3] = b0.w;
            b.v[4] = b1.x; b.v[5] = b1.y; b.v[6] = b1.z; b.v[7] = b1.w;
            acc = acc + b;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) store_fr(out, blockIdx.x, acc);
}

void k_poly_eval_sets(const EvalSet *sets, int nsets, uint64_t n, DevBuf &scratch, hipStream_t s) {
    int total = 0;
    for (int k = 0; k < nsets; k++) total += std::max(sets[k].np, 0);
    if (total == 0) return;
    const uint32_t nb = (uint32_t)std::max<uint64_t>(1, (n + 256 * EV_K - 1) / (256 * EV_K));
    // layout: [partials total*nb][results total]: every group of up to 8 polys
    // has its own slice, so all launch back to back and ONE copy and ONE
    // synchronisation return every value (round 5 evaluates 18 polys at two
    // points: four host round trips before)
    size_t need = (size_t)total * nb * 32 + (size_t)total * 32 + 64;
    if (scratch.bytes < need) scratch.alloc(need);
    uint64_t *partial = scratch.u64();
    uint64_t *res = partial + (size_t)total * nb * 4;
    int q = 0;  // polys launched so far
    for (int k = 0; k < nsets; k++) {
        const Fr &x = sets[k].x;
        const Fr x256 = pow_u64(x, 256), xblk = pow_u64(x, 256ull * EV_K);
        for (int p0 = 0; p0 < sets[k].np; p0 += 8) {
            const int np = std::min(sets[k].np - p0, 8);
            EvalPtrs ptrs = {};
            for (int j = 0; j < np; j++) ptrs.p[j] = sets[k].polys[p0 + j];
            uint64_t *pt = partial + (size_t)q * nb * 4;
            switch (np) {
#define PNP_EV(K)                                                                                 \
    case K:                                                                                       \
        hipLaunchKernelGGL(k_eval_partial<K>, dim3(nb), dim3(256), 0, s, ptrs, n, x, x256, xblk, pt); \
        break;
                PNP_EV(1) PNP_EV(2) PNP_EV(3) PNP_EV(4) PNP_EV(5) PNP_EV(6) PNP_EV(7) PNP_EV(8)
#undef PNP_EV
            }
            PNP_HIP(hipGetLastError());
            hipLaunchKernelGGL(k_sum_partials, dim3(np), dim3(256), 0, s, pt, (uint64_t)nb, res + 4 * q);
            PNP_HIP(hipGetLastError());
            q += np;
        }
    }
    std::vector<Fr> host((size_t)total);
    PNP_HIP(hipMemcpyAsync(host.data(), res, 32 * (size_t)total, hipMemcpyDeviceToHost, s));
    PNP_HIP(hipStreamSynchronize(s));
    q = 0;
    for (int k = 0; k < nsets; k++)
        for (int p = 0; p < sets[k].np; p++) sets[k].out[p] = host[q++];
}

void k_poly_eval_multi(const uint64_t *const *polys, int npolys, uint64_t n, const Fr &x,
                       DevBuf &scratch, Fr *out, hipStream_t s) {
    const EvalSet set = {polys, npolys, x, out};
    k_poly_eval_sets(&set, 1, n, scratch, s);
}

void k_poly_eval(const uint64_t *d, uint64_t n, const Fr &x, DevBuf &scratch, Fr *out,
                 hipStream_t s) {
    const uint64_t *p[1] = {d};
    k_poly_eval_multi(p, 1, n, x, scratch, out, s);
}

// ---------------------------------------------------------------- geometric fill
// d[i] = c0 * r^i — coefficient form of a scaled Lagrange basis polynomial:
// iNTT(v * e_pos)_j = v n^-1 w^(-pos j), so L1 / PI coefficients need no NTT
__global__ void k_geometric_(uint64_t *d, uint64_t n, Fr c0, Fr r, uint32_t chunk) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t lo = t * chunk;
    if (lo >= n) return;
    uint64_t hi = lo + chunk < n ? lo + chunk : n;
    Fr v = c0 * pow_u64(r, lo);
    for (uint64_t i = lo; i < hi; i++) {
        store_fr(d, i, v);
        v = v * r;
    }
}
void k_geometric(uint64_t *d, uint64_t n, const Fr &c0, const Fr &r, hipStream_t s) {
    if (!n) return;
    const uint32_t chunk = 16;
    hipLaunchKernelGGL(k_geometric_, dim3(nblk((n + chunk - 1) / chunk)), dim3(256), 0, s, d, n, c0,
                       r, chunk);
    PNP_HIP(hipGetLastError());
}

// ---------------------------------------------------------------- synthetic inputs
__device__ __forceinline__ uint64_t splitmix(uint64_t x) {
    x += 0x9e3779b97f4a7c15ULL;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
    return x ^ (x >> 31);
}
__global__ void k_random_fr_(uint64_t *d, uint64_t n, uint64_t seed) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    Fr r;
    uint64_t h = seed * 0x2545F4914F6CDD1DULL + i * 4;
    for (int k = 0; k < 4; k++) {
        uint64_t w = splitmix(h + k);
        r.v[2 * k] = (uint32_t)w;
        r.v[2 * k + 1] = (uint32_t)(w >> 32);
    }
    r.v[7] &= 0x7fffffffu;  // < 2^255 < 2r
    reduce_once(r);
    store_fr(d, i, r);  // uniform-ish canonical value used directly as a Montgomery residue
}
void k_random_fr(uint64_t *d, uint64_t n, uint64_t seed, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_random_fr_, dim3(nblk(n)), dim3(256), 0, s, d, n, seed);
    PNP_HIP(hipGetLastError());
}

// d[i] += c z^(len-1-i), i < len: the carry of a polynomial division by
// (X - z) split over coefficient ranges (the part above this range)
// Thread t of T owns the elements t, t + T, t + 2T, ... (coalesced across a
// wave) and walks them from the top down: c z^(len-1-i) for the top one by a
// product of the powers z^(2^k) (kernel arguments, no squaring chain per
// thread), then one product by z^T per step.  (The contiguous 64-element
// chunks of one thread each took ~90 dependent products on 128 waves: ~85 us
// per launch, exposed at 8 ranks.)
struct ZPow {
    Fr p[32];  // z^(2^k)
};
__global__ void k_add_powers_(uint64_t *d, uint64_t len, Fr c, ZPow zp, Fr zT, uint64_t T) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (t >= T || t >= len) return;
    uint64_t i = t + (len - 1 - t) / T * T;  // this thread's top element
    uint64_t e = len - 1 - i;
    Fr p = c;
    for (int k = 0; e; k++, e >>= 1)
        if (e & 1) p = p * zp.p[k];
    for (;; i -= T) {
        store_fr(d, i, load_fr(d, i) + p);
        if (i < T) break;
        p = p * zT;
    }
}
void k_add_powers(uint64_t *d, uint64_t len, const Fr &c, const Fr &z, hipStream_t s) {
    if (!len) return;
    if (len >= (1ull << 32)) {
        set_error("k_add_powers: length %llu", (unsigned long long)len);
        throw Error(PNP_E_ARG);
    }
    const uint64_t T = std::min<uint64_t>(len, 1u << 16);  // <= 8 elements a thread at 2^19
    ZPow zp;
    zp.p[0] = z;
    for (int k = 1; k < 32; k++) zp.p[k] = zp.p[k - 1] * zp.p[k - 1];
    hipLaunchKernelGGL(k_add_powers_, dim3(nblk(T)), dim3(256), 0, s, d, len, c, zp, pow_u64(z, T), T);
    PNP_HIP(hipGetLastError());
}

}  // namespace pnp
