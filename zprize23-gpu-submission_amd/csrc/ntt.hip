// ntt.hip — radix-2 NTT over BLS12-381 Fr for gfx950.
//
// Semantics: natural order in and out, omega_N = ROOT32^(2^(32-lg)), inverse
// scaled by N^-1, coset generator g = 7 (forward: x_i *= g^i first, inverse:
// x_i *= g^-i last) — the reference's Ntt/Intt/Ntt_coset/Intt_coset
// (utils/function.cu:249-273 -> zksnark_ntt.cu:74-92 -> ntt_kernel/ntt.cuh:57-144).
//
// Design (MI355X-first, not the reference's CT kernels):
//   * Decimation-in-frequency passes of K levels each over LDS tiles of 1024
//     elements (32 KiB, four workgroups per CU).  A tile holds G = 1024/2^K
//     interleaved sub-transforms so every global row access is G consecutive
//     32-byte elements (G*32 B contiguous).  LDS keeps the element split in two
//     16-byte planes so each lane's ds_read_b128 / ds_write_b128 is
//     conflict-free.
//   * Twiddles w_N^e come from a per-size table (computed once per context,
//     HBM-resident; its hot part lives in L2/MALL).
//   * The DIF output is bit-reversed; one in-place tiled pass (32x32 tiles,
//     tile pairs swapped through LDS) restores natural order and fuses the
//     N^-1 and g^-i scalings of the inverse / coset-inverse transforms.
#include "pnp_internal.h"
#include "fr29.cuh"

namespace pnp {

#ifndef PNP_NTT_LGTILE
#define PNP_NTT_LGTILE 10
#endif
static constexpr int LGTILE = PNP_NTT_LGTILE;  // elements per LDS tile = levels per pass (max)
static constexpr int TILE = 1 << LGTILE;
#ifndef PNP_NTT_THREADS
#define PNP_NTT_THREADS 512
#endif
static constexpr int NTT_THREADS = PNP_NTT_THREADS;

// ---------------------------------------------------------------- tables
__global__ void k_powers_table(uint64_t *out, uint64_t count, Fr base, uint32_t chunk) {
    uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t start = t * chunk;
    if (start >= count) return;
    Fr p = pow_u64(base, start);
    uint64_t end = start + chunk < count ? start + chunk : count;
    for (uint64_t i = start; i < end; i++) {
        store_fr(out, i, p);
        p = p * base;
    }
}

static Fr host_root(uint32_t lg) {
    const uint64_t root32[4] = {13381757501831005802ULL, 6564924994866501612ULL,
                                789602057691799140ULL, 6625830629041353339ULL};
    Fr r = from_u64_limbs<FrP>(root32);
    return pow_u64(r, 1ULL << (32 - lg));
}
static Fr host_gen() {
    Fr seven = Fr::zero();
    seven.v[0] = 7;
    return to_mont(seven);
}

static void powers_table(DevBuf &buf, uint64_t count, const Fr &base, hipStream_t s) {
    buf.alloc(count * 32);
    const uint32_t chunk = 64;
    uint64_t threads = (count + chunk - 1) / chunk;
    uint32_t blocks = (uint32_t)((threads + 255) / 256);
    hipLaunchKernelGGL(k_powers_table, dim3(blocks), dim3(256), 0, s, buf.u64(), count, base, chunk);
    PNP_HIP(hipGetLastError());
}

const uint64_t *ntt_twiddles(NttTables &t, uint32_t lg, bool inverse, hipStream_t s) {
    auto &m = inverse ? t.inv : t.fwd;
    auto it = m.find(lg);
    if (it != m.end()) return it->second.u64();
    Fr w = host_root(lg);
    if (inverse) w = pnp::inverse(w);
    DevBuf buf;
    uint64_t half = lg ? (1ULL << (lg - 1)) : 1;
    powers_table(buf, half, w, s);
    const uint64_t *p = buf.u64();
    m.emplace(lg, std::move(buf));
    return p;
}

// Twiddle rows.  A level of a pass reads w_N^(r 2^sh),
// r = j + mlow 2^lg_hlo, sh = lg_N - 1 - lg_hlo - l: from the plain table every
// 2^sh-th entry, i.e. one 32-B twiddle per 128-B line once sh >= 2 (the first
// DIF pass of a block LDE fetched ~62 B of twiddle lines per element,
// profiles/r05_ntt_pmc_traffic.txt).  Row sh holds exactly those entries,
// densely: rows[N - N / 2^sh + r] = w_N^(r 2^sh), so a tile's G consecutive
// columns read G consecutive twiddles of every level.  N - 1 entries per size
// and direction (2x the plain table).  PNP_NTT_ROWS=0: the plain table
__global__ void k_twiddle_rows(const uint64_t *tw, uint32_t lg, uint64_t *rows) {
    const uint64_t N = 1ULL << lg;
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;  // position in rows, < N - 1
    if (i >= N - 1) return;
    // row sh starts at N - N / 2^sh: sh = the number of leading ones of i in lg bits
    uint32_t sh = 0;
    while (i >= N - (N >> (sh + 1))) sh++;
    const uint64_t r = i - (N - (N >> sh));
    const uint4 *src = reinterpret_cast<const uint4 *>(tw + 4 * (r << sh));
    uint4 *dst = reinterpret_cast<uint4 *>(rows + 4 * i);
    dst[0] = src[0];
    dst[1] = src[1];
}

static bool ntt_rows_enabled() {
    static const bool on = [] {
        const char *e = getenv("PNP_NTT_ROWS");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

static const uint64_t *ntt_twiddle_rows(NttTables &t, uint32_t lg, bool inverse, hipStream_t s) {
    auto &m = inverse ? t.inv_rows : t.fwd_rows;
    auto it = m.find(lg);
    if (it != m.end()) return it->second.u64();
    const uint64_t *tw = ntt_twiddles(t, lg, inverse, s);
    const uint64_t cnt = (1ULL << lg) - 1;
    DevBuf buf(std::max<uint64_t>(cnt, 1) * 32);
    hipLaunchKernelGGL(k_twiddle_rows, dim3((uint32_t)((cnt + 255) / 256)), dim3(256), 0, s, tw, lg, buf.u64());
    PNP_HIP(hipGetLastError());
    const uint64_t *p = buf.u64();
    m.emplace(lg, std::move(buf));
    return p;
}

// a 2^256-form table (32-bit Montgomery Fr) -> its 2^261 form in radix 2^29
__global__ void k_table_to_r29(const uint64_t *tab, uint64_t count, uint32_t *out) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= count) return;
    const uint32_t *w = reinterpret_cast<const uint32_t *>(tab + 4 * i);
    R29 c;
#pragma unroll
    for (int k = 0; k < 9; k++) c.l[k] = R29_C266[k];
    const R29 x = r29_canon(r29_mul(r29_from_words(w), c));
    uint32_t *o = out + 9 * i;
#pragma unroll
    for (int k = 0; k < 9; k++) o[k] = x.l[k];
}

static const uint32_t *to_r29_table(std::map<uint32_t, DevBuf> &m, uint32_t key, const uint64_t *tab,
                                    uint64_t count, hipStream_t s) {
    auto it = m.find(key);
    if (it != m.end()) return static_cast<const uint32_t *>(it->second.p);
    DevBuf buf(count * 36);
    hipLaunchKernelGGL(k_table_to_r29, dim3((uint32_t)((count + 255) / 256)), dim3(256), 0, s, tab, count,
                       static_cast<uint32_t *>(buf.p));
    PNP_HIP(hipGetLastError());
    const uint32_t *p = static_cast<const uint32_t *>(buf.p);
    m.emplace(key, std::move(buf));
    return p;
}

static const uint32_t *ntt_twiddles29(NttTables &t, uint32_t lg, bool inverse, hipStream_t s) {
    const uint64_t half = lg ? (1ULL << (lg - 1)) : 1;
    return to_r29_table(inverse ? t.inv29 : t.fwd29, lg, ntt_twiddles(t, lg, inverse, s), half, s);
}

void ntt_prepare_coset(NttTables &t, hipStream_t s) {
    if (t.coset_ready) return;
    Fr g = host_gen();
    Fr gi = pnp::inverse(g);
    powers_table(t.coset_lo, 4096, g, s);
    powers_table(t.coset_hi, 1 << 14, pow_u64(g, 4096), s);
    powers_table(t.coset_inv_lo, 4096, gi, s);
    powers_table(t.coset_inv_hi, 1 << 14, pow_u64(gi, 4096), s);
    t.coset_ready = true;
}

__device__ __forceinline__ Fr coset_pow(const uint64_t *hi, const uint64_t *lo, uint64_t i) {
    return load_fr(hi, i >> 12) * load_fr(lo, i & 4095);
}

// ---------------------------------------------------------------- DIF / DIT pass
// One pass = K levels with half sizes H_lo*2^(K-1) ... H_lo over tiles of
// TILE elements (G = TILE >> K interleaved sub-transforms per tile).
// DIF (natural in, bit-reversed out): levels from the largest half size down,
// butterfly (a + b, (a - b) w).  DIT (bit-reversed in, natural out): levels
// from the smallest half size up, butterfly (a + b w, a - b w), same twiddles.
// Optional fusions: `src` + `pre` (load src[idx & src_mask] * pre[idx] instead
// of data[idx]: the coset twist of an LDE in its first pass) and `post` (store
// x * post[idx]: the block twist after the last inverse pass).
template <int K, bool DIT>
__global__ __launch_bounds__(NTT_THREADS) void k_ntt_pass(uint64_t *data, const uint64_t *tw,
                                                           uint32_t lg_n, uint32_t lg_hlo,
                                                           const uint64_t *src, const uint64_t *pre,
                                                           uint64_t src_mask, const uint64_t *post) {
    constexpr int G = TILE >> K;
    __shared__ uint4 lds_lo[TILE];
    __shared__ uint4 lds_hi[TILE];
    const uint64_t hlo = 1ULL << lg_hlo;
    const uint64_t gid0 = (uint64_t)blockIdx.x * G;
    // load: element (m, g) of the tile -> lds[m*G + g]
    for (int e = threadIdx.x; e < TILE; e += NTT_THREADS) {
        int g = e % G, m = e / G;
        uint64_t gid = gid0 + g;
        uint64_t j = gid & (hlo - 1), b = gid >> lg_hlo;
        uint64_t idx = (b << (lg_hlo + K)) + j + ((uint64_t)m << lg_hlo);
        if (src) {
            Fr x = load_fr(src, idx & src_mask);
            if (pre) x = x * load_fr(pre, idx);
            lds_lo[e] = make_uint4(x.v[0], x.v[1], x.v[2], x.v[3]);
            lds_hi[e] = make_uint4(x.v[4], x.v[5], x.v[6], x.v[7]);
        } else {
            const uint4 *p = reinterpret_cast<const uint4 *>(data + 4 * idx);
            lds_lo[e] = p[0];
            lds_hi[e] = p[1];
        }
    }
    __syncthreads();
    for (int step = 0; step < K; step++) {
        const int l = DIT ? step : K - 1 - step;
        const uint32_t sh = lg_n - 1 - lg_hlo - l;
        // half size 1: every twiddle is w^0 = 1 (uniform branch, no product)
        const bool unit = lg_hlo == 0 && l == 0;
        for (int bf = threadIdx.x; bf < TILE / 2; bf += NTT_THREADS) {
            int g = bf % G, q = bf / G;
            int mlow = q & ((1 << l) - 1);
            int m = ((q >> l) << (l + 1)) | mlow;
            int e0 = m * G + g, e1 = (m + (1 << l)) * G + g;
            uint64_t gid = gid0 + g;
            uint64_t j = gid & (hlo - 1);
            uint64_t r = j + ((uint64_t)mlow << lg_hlo);
            uint4 a0 = lds_lo[e0], a1 = lds_hi[e0], b0 = lds_lo[e1], b1 = lds_hi[e1];
            Fr a, b;
            a.v[0] = a0.x; a.v[1] = a0.y; a.v[2] = a0.z; a.v[3] = a0.w;
            a.v[4] = a1.x; a.v[5] = a1.y; a.v[6] = a1.z; a.v[7] = a1.w;
            b.v[0] = b0.x; b.v[1] = b0.y; b.v[2] = b0.z; b.v[3] = b0.w;
            b.v[4] = b1.x; b.v[5] = b1.y; b.v[6] = b1.z; b.v[7] = b1.w;
            Fr s, d;
            if (unit) {
                s = a + b;
                d = a - b;
            } else if (DIT) {
                Fr t = b * load_fr(tw, r << sh);
                s = a + t;
                d = a - t;
            } else {
                s = a + b;
                d = (a - b) * load_fr(tw, r << sh);
            }
            lds_lo[e0] = make_uint4(s.v[0], s.v[1], s.v[2], s.v[3]);
            lds_hi[e0] = make_uint4(s.v[4], s.v[5], s.v[6], s.v[7]);
            lds_lo[e1] = make_uint4(d.v[0], d.v[1], d.v[2], d.v[3]);
            lds_hi[e1] = make_uint4(d.v[4], d.v[5], d.v[6], d.v[7]);
        }
        __syncthreads();
    }
    for (int e = threadIdx.x; e < TILE; e += NTT_THREADS) {
        int g = e % G, m = e / G;
        uint64_t gid = gid0 + g;
        uint64_t j = gid & (hlo - 1), b = gid >> lg_hlo;
        uint64_t idx = (b << (lg_hlo + K)) + j + ((uint64_t)m << lg_hlo);
        if (post) {
            uint4 lo = lds_lo[e], hi = lds_hi[e];
            Fr x;
            x.v[0] = lo.x; x.v[1] = lo.y; x.v[2] = lo.z; x.v[3] = lo.w;
            x.v[4] = hi.x; x.v[5] = hi.y; x.v[6] = hi.z; x.v[7] = hi.w;
            store_fr(data, idx, x * load_fr(post, idx));
        } else {
            uint4 *dst = reinterpret_cast<uint4 *>(data + 4 * idx);
            dst[0] = lds_lo[e];
            dst[1] = lds_hi[e];
        }
    }
}

// The same pass with two levels per LDS round trip (radix-4 groups): each of
// 256 lanes reads 4 elements, does the 4 butterflies of two consecutive
// levels in registers (3 twiddles) and writes 4 elements back, so the tile
// makes half the LDS round trips and barriers of k_ntt_pass; an odd K ends
// (DIF) or ends (DIT) with one radix-2 level.  Same indexing and twiddles as
// k_ntt_pass (level l, group element m: pair distance 2^l in m).
#ifndef PNP_NTT4_THREADS
#define PNP_NTT4_THREADS 256
#endif
constexpr int NTT4_THREADS = PNP_NTT4_THREADS;
__device__ __forceinline__ Fr lds_get(const uint4 *lo, const uint4 *hi, int e) {
    const uint4 a = lo[e], b = hi[e];
    Fr x;
    x.v[0] = a.x; x.v[1] = a.y; x.v[2] = a.z; x.v[3] = a.w;
    x.v[4] = b.x; x.v[5] = b.y; x.v[6] = b.z; x.v[7] = b.w;
    return x;
}
__device__ __forceinline__ void lds_put(uint4 *lo, uint4 *hi, int e, const Fr &x) {
    lo[e] = make_uint4(x.v[0], x.v[1], x.v[2], x.v[3]);
    hi[e] = make_uint4(x.v[4], x.v[5], x.v[6], x.v[7]);
}
// Lazy residues inside a radix-4 tile: values stay in [0, 2r) between the
// levels of a pass and are made canonical when the pass stores them.  The
// twiddle products skip their final subtraction (a < 2r, w < r: result
// < r (2r / 2^256 + 1) < 2r); sums and differences stay in [0, 2r) with one
// conditional step each, as before.  (2r < 2^256 but 4r is not: r = 0.45 *
// 2^256, so Harvey's unconditional a - b + 2r does not fit 8 limbs.)
constexpr uint32_t FR_2R[8] = {PNP_LIMB(0xfffffffe00000002), PNP_LIMB(0xa77b4805fffcb7fd),
                               PNP_LIMB(0x6673b0101343b00a), PNP_LIMB(0xe7db4ea6533afa90)};
__device__ __forceinline__ Fr lz_add(const Fr &a, const Fr &b) {  // [0, 2r) + [0, 2r) -> [0, 2r)
    Fr s, t;
    const uint32_t c = add_n<8>(s.v, a.v, b.v);  // < 4r < 2^257: carry out possible
    const uint32_t br = sub_n<8>(t.v, s.v, FR_2R);
    const bool keep = br && !c;                  // s < 2r
#pragma unroll
    for (int i = 0; i < 8; i++) s.v[i] = keep ? s.v[i] : t.v[i];
    return s;
}
__device__ __forceinline__ Fr lz_sub(const Fr &a, const Fr &b) {  // [0, 2r) - [0, 2r) -> [0, 2r)
    Fr d, t;
    const uint32_t br = sub_n<8>(d.v, a.v, b.v);
    add_n<8>(t.v, d.v, FR_2R);
#pragma unroll
    for (int i = 0; i < 8; i++) d.v[i] = br ? t.v[i] : d.v[i];
    return d;
}
__device__ __forceinline__ Fr lz_mul(const Fr &a, const Fr &w) {  // a < 2r, w < r -> [0, 2r)
#ifdef __HIP_DEVICE_COMPILE__
    return mont_mul_dev<FrP, false>(a, w);
#else
    return a * w;  // (host pass of the single-source compile; never called)
#endif
}
__device__ __forceinline__ Fr lz_canon(Fr a) {  // [0, 2r) -> [0, r)
    reduce_once(a);
    return a;
}

template <int K, bool DIT>
__global__ __launch_bounds__(NTT4_THREADS) void k_ntt_pass4(uint64_t *data, const uint64_t *tw,
                                                            uint32_t lg_n, uint32_t lg_hlo,
                                                            const uint64_t *src, const uint64_t *pre,
                                                            uint64_t src_mask, const uint64_t *post,
                                                            int rows = 0) {
    constexpr int G = TILE >> K;
    __shared__ uint4 lds_lo[TILE];
    __shared__ uint4 lds_hi[TILE];
    const uint64_t hlo = 1ULL << lg_hlo;
    const uint64_t gid0 = (uint64_t)blockIdx.x * G;
    for (int e = threadIdx.x; e < TILE; e += NTT4_THREADS) {
        const int g = e % G, m = e / G;
        const uint64_t gid = gid0 + g;
        const uint64_t j = gid & (hlo - 1), b = gid >> lg_hlo;
        const uint64_t idx = (b << (lg_hlo + K)) + j + ((uint64_t)m << lg_hlo);
        if (src) {
            Fr x = load_fr(src, idx & src_mask);
            if (pre) x = lz_mul(x, load_fr(pre, idx));  // [0, 2r): the tile is lazy
            lds_put(lds_lo, lds_hi, e, x);
        } else {
            const uint4 *p = reinterpret_cast<const uint4 *>(data + 4 * idx);
            lds_lo[e] = p[0];
            lds_hi[e] = p[1];
        }
    }
    __syncthreads();
    // twiddle of a level-l butterfly whose lower element has low bits mlow
    // (rows: the dense row of its shift, ntt_twiddle_rows)
    auto twl = [&](uint64_t j, int l, uint32_t mlow) {
        const uint32_t sh = lg_n - 1 - lg_hlo - l;
        const uint64_t r = j + ((uint64_t)mlow << lg_hlo);
        return rows ? load_fr(tw, (1ULL << lg_n) - (1ULL << (lg_n - sh)) + r) : load_fr(tw, r << sh);
    };
    constexpr int NPAIR = K / 2;
#pragma unroll 1
    for (int pr = 0; pr < NPAIR; pr++) {
        // DIF: levels (hi, hi - 1) from K - 1 down; DIT: (lo, lo + 1) from 0 up
        const int l = DIT ? 2 * pr : K - 1 - 2 * pr;  // the first level of the pair
        const int lb = DIT ? l : l - 1;                // the lower of the two
        for (int q = threadIdx.x; q < TILE / 4; q += NTT4_THREADS) {
            const int g = q % G, q4 = q / G;
            const uint32_t ml = q4 & ((1 << lb) - 1);
            const int m = ((q4 >> lb) << (lb + 2)) | (int)ml;
            const int e0 = m * G + g, e1 = (m + (1 << lb)) * G + g, e2 = (m + (2 << lb)) * G + g,
                      e3 = (m + (3 << lb)) * G + g;
            const uint64_t j = (gid0 + g) & (hlo - 1);
            Fr x0 = lds_get(lds_lo, lds_hi, e0), x1 = lds_get(lds_lo, lds_hi, e1);
            Fr x2 = lds_get(lds_lo, lds_hi, e2), x3 = lds_get(lds_lo, lds_hi, e3);
            const bool unit = lg_hlo == 0 && lb == 0;  // level lb has half size 1
            // (lazy residues in [0, 2r), see lz_add)
            if (DIT) {
                // level lb: (x0, x1), (x2, x3), one twiddle
                if (unit) {
                    Fr t = x1; x1 = lz_sub(x0, t); x0 = lz_add(x0, t);
                    t = x3; x3 = lz_sub(x2, t); x2 = lz_add(x2, t);
                } else {
                    const Fr w = twl(j, lb, ml);
                    Fr t = lz_mul(x1, w); x1 = lz_sub(x0, t); x0 = lz_add(x0, t);
                    t = lz_mul(x3, w); x3 = lz_sub(x2, t); x2 = lz_add(x2, t);
                }
                // level lb + 1: (x0, x2) with low bits ml, (x1, x3) with ml + 2^lb
                Fr t = lz_mul(x2, twl(j, lb + 1, ml)); x2 = lz_sub(x0, t); x0 = lz_add(x0, t);
                t = lz_mul(x3, twl(j, lb + 1, ml + (1u << lb))); x3 = lz_sub(x1, t); x1 = lz_add(x1, t);
            } else {
                // level lb + 1: (x0, x2) with low bits ml, (x1, x3) with ml + 2^lb
                Fr d = lz_mul(lz_sub(x0, x2), twl(j, lb + 1, ml)); x0 = lz_add(x0, x2); x2 = d;
                d = lz_mul(lz_sub(x1, x3), twl(j, lb + 1, ml + (1u << lb))); x1 = lz_add(x1, x3); x3 = d;
                // level lb: (x0, x1), (x2, x3)
                if (unit) {
                    d = lz_sub(x0, x1); x0 = lz_add(x0, x1); x1 = d;
                    d = lz_sub(x2, x3); x2 = lz_add(x2, x3); x3 = d;
                } else {
                    const Fr w = twl(j, lb, ml);
                    d = lz_mul(lz_sub(x0, x1), w); x0 = lz_add(x0, x1); x1 = d;
                    d = lz_mul(lz_sub(x2, x3), w); x2 = lz_add(x2, x3); x3 = d;
                }
            }
            lds_put(lds_lo, lds_hi, e0, x0);
            lds_put(lds_lo, lds_hi, e1, x1);
            lds_put(lds_lo, lds_hi, e2, x2);
            lds_put(lds_lo, lds_hi, e3, x3);
        }
        __syncthreads();
    }
    if (K & 1) {  // the remaining level: DIF level 0, DIT level K - 1
        const int l = DIT ? K - 1 : 0;
        const bool unit = lg_hlo == 0 && l == 0;
        for (int bf = threadIdx.x; bf < TILE / 2; bf += NTT4_THREADS) {
            const int g = bf % G, q = bf / G;
            const int mlow = q & ((1 << l) - 1);
            const int m = ((q >> l) << (l + 1)) | mlow;
            const int e0 = m * G + g, e1 = (m + (1 << l)) * G + g;
            const uint64_t j = (gid0 + g) & (hlo - 1);
            Fr a = lds_get(lds_lo, lds_hi, e0), b = lds_get(lds_lo, lds_hi, e1), s2, d;
            if (unit) {
                s2 = lz_add(a, b);
                d = lz_sub(a, b);
            } else if (DIT) {
                const Fr t = lz_mul(b, twl(j, l, (uint32_t)mlow));
                s2 = lz_add(a, t);
                d = lz_sub(a, t);
            } else {
                s2 = lz_add(a, b);
                d = lz_mul(lz_sub(a, b), twl(j, l, (uint32_t)mlow));
            }
            lds_put(lds_lo, lds_hi, e0, s2);
            lds_put(lds_lo, lds_hi, e1, d);
        }
        __syncthreads();
    }
    for (int e = threadIdx.x; e < TILE; e += NTT4_THREADS) {
        const int g = e % G, m = e / G;
        const uint64_t gid = gid0 + g;
        const uint64_t j = gid & (hlo - 1), b = gid >> lg_hlo;
        const uint64_t idx = (b << (lg_hlo + K)) + j + ((uint64_t)m << lg_hlo);
        // canonical out: the reducing product (x < 2r, post < r) or one subtraction
        if (post)
            store_fr(data, idx, lds_get(lds_lo, lds_hi, e) * load_fr(post, idx));
        else
            store_fr(data, idx, lz_canon(lds_get(lds_lo, lds_hi, e)));
    }
}

// The same pass in radix-2^29 arithmetic (fr29.cuh): canonical 2^256-form Fr
// in and out (the HBM layout is unchanged), nine-limb values in LDS (two
// 16-byte planes + one 4-byte plane, 36 KiB per tile), twiddles / twists from
// the 2^261-form tables.  Bounds (tests/test_fr29.py): a DIF level l of the
// pass doubles the inputs (< 2^l 1.04 r), its difference adds 2^(l+1) r; a DIT
// level adds a product output (< 4 r) and 4 r; outputs < 2^264 -> r29_canon.
template <int K, bool DIT>
__global__ __launch_bounds__(NTT_THREADS) void k_ntt_pass29(uint64_t *data, const uint32_t *tw,
                                                             uint32_t lg_n, uint32_t lg_hlo,
                                                             const uint64_t *src, const uint32_t *pre,
                                                             uint64_t src_mask, const uint32_t *post) {
    constexpr int G = TILE >> K;
    __shared__ uint4 l_lo[TILE];
    __shared__ uint4 l_mid[TILE];
    __shared__ uint32_t l_top[TILE];
    auto put = [&](int e, const R29 &x) {
        l_lo[e] = make_uint4(x.l[0], x.l[1], x.l[2], x.l[3]);
        l_mid[e] = make_uint4(x.l[4], x.l[5], x.l[6], x.l[7]);
        l_top[e] = x.l[8];
    };
    auto get = [&](int e) {
        const uint4 a = l_lo[e], b = l_mid[e];
        R29 x;
        x.l[0] = a.x; x.l[1] = a.y; x.l[2] = a.z; x.l[3] = a.w;
        x.l[4] = b.x; x.l[5] = b.y; x.l[6] = b.z; x.l[7] = b.w;
        x.l[8] = l_top[e];
        return x;
    };
    const uint64_t hlo = 1ULL << lg_hlo;
    const uint64_t gid0 = (uint64_t)blockIdx.x * G;
    for (int e = threadIdx.x; e < TILE; e += NTT_THREADS) {
        const int g = e % G, m = e / G;
        const uint64_t gid = gid0 + g;
        const uint64_t j = gid & (hlo - 1), b = gid >> lg_hlo;
        const uint64_t idx = (b << (lg_hlo + K)) + j + ((uint64_t)m << lg_hlo);
        const uint4 *p = reinterpret_cast<const uint4 *>((src ? src + 4 * (idx & src_mask) : data + 4 * idx));
        const uint4 q0 = p[0], q1 = p[1];
        const uint32_t w[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
        R29 x = r29_from_words(w);
        if (src) x = r29_mul(x, r29_load(pre, idx));
        put(e, x);
    }
    __syncthreads();
#pragma unroll 1
    for (int step = 0; step < K; step++) {
        const int l = DIT ? step : K - 1 - step;
        const uint32_t sh = lg_n - 1 - lg_hlo - l;
        const bool unit = lg_hlo == 0 && l == 0;  // half size 1: twiddle 1, no product
        const uint32_t *kd = R29_KDIF[step];
        for (int bf = threadIdx.x; bf < TILE / 2; bf += NTT_THREADS) {
            const int g = bf % G, q = bf / G;
            const int mlow = q & ((1 << l) - 1);
            const int m = ((q >> l) << (l + 1)) | mlow;
            const int e0 = m * G + g, e1 = (m + (1 << l)) * G + g;
            const uint64_t j = (gid0 + g) & (hlo - 1);
            const uint64_t r = j + ((uint64_t)mlow << lg_hlo);
            const R29 a = get(e0), b = get(e1);
            R29 s, d;
            if (DIT) {
                const R29 t = unit ? b : r29_mul(b, r29_load(tw, r << sh));
                s = r29_add(a, t);
                d = r29_sub(a, t, R29_KDIT);
            } else {
                s = r29_add(a, b);
                d = r29_sub(a, b, kd);
                if (!unit) d = r29_mul(d, r29_load(tw, r << sh));
            }
            put(e0, s);
            put(e1, d);
        }
        __syncthreads();
    }
    for (int e = threadIdx.x; e < TILE; e += NTT_THREADS) {
        const int g = e % G, m = e / G;
        const uint64_t gid = gid0 + g;
        const uint64_t j = gid & (hlo - 1), b = gid >> lg_hlo;
        const uint64_t idx = (b << (lg_hlo + K)) + j + ((uint64_t)m << lg_hlo);
        R29 x = get(e);
        if (post) x = r29_mul(x, r29_load(post, idx));
        x = r29_canon(x);
        uint32_t w[8];
        r29_to_words(x, w);
        uint4 *dst = reinterpret_cast<uint4 *>(data + 4 * idx);
        dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
        dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
    }
}

// The radix-2^29 pass with two levels per LDS round trip (radix-4 groups as
// k_ntt_pass4, arithmetic as k_ntt_pass29).  Every element meets exactly the
// operations of k_ntt_pass29 in the same order — level by level, the same
// lifted constant R29_KDIF[step] for the differences of step `step`, the same
// twiddle products — so the bounds tests/test_fr29.py asserts for that pass
// hold here unchanged.  Per butterfly the radix-2^29 product (153 bare
// multiply-adds, no carry instructions, no hazard s_nops) issues ~20% fewer
// VALU cycles than the 32-bit one (256 multiply-adds and carries); the radix-4
// grouping halves the LDS round trips of the nine-limb planes.
template <int K, bool DIT>
__global__ __launch_bounds__(NTT4_THREADS) void k_ntt_pass4_29(uint64_t *data, const uint32_t *tw,
                                                                uint32_t lg_n, uint32_t lg_hlo,
                                                                const uint64_t *src, const uint32_t *pre,
                                                                uint64_t src_mask, const uint32_t *post) {
    constexpr int G = TILE >> K;
    __shared__ uint4 l_lo[TILE];
    __shared__ uint4 l_mid[TILE];
    __shared__ uint32_t l_top[TILE];
    auto put = [&](int e, const R29 &x) {
        l_lo[e] = make_uint4(x.l[0], x.l[1], x.l[2], x.l[3]);
        l_mid[e] = make_uint4(x.l[4], x.l[5], x.l[6], x.l[7]);
        l_top[e] = x.l[8];
    };
    auto get = [&](int e) {
        const uint4 a = l_lo[e], b = l_mid[e];
        R29 x;
        x.l[0] = a.x; x.l[1] = a.y; x.l[2] = a.z; x.l[3] = a.w;
        x.l[4] = b.x; x.l[5] = b.y; x.l[6] = b.z; x.l[7] = b.w;
        x.l[8] = l_top[e];
        return x;
    };
    const uint64_t hlo = 1ULL << lg_hlo;
    const uint64_t gid0 = (uint64_t)blockIdx.x * G;
    for (int e = threadIdx.x; e < TILE; e += NTT4_THREADS) {
        const int g = e % G, m = e / G;
        const uint64_t gid = gid0 + g;
        const uint64_t j = gid & (hlo - 1), b = gid >> lg_hlo;
        const uint64_t idx = (b << (lg_hlo + K)) + j + ((uint64_t)m << lg_hlo);
        const uint4 *p = reinterpret_cast<const uint4 *>((src ? src + 4 * (idx & src_mask) : data + 4 * idx));
        const uint4 q0 = p[0], q1 = p[1];
        const uint32_t w[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
        R29 x = r29_from_words(w);
        if (src && pre) x = r29_mul(x, r29_load(pre, idx));
        put(e, x);
    }
    __syncthreads();
    auto twl = [&](uint64_t j, int l, uint32_t mlow) {
        return r29_load(tw, (j + ((uint64_t)mlow << lg_hlo)) << (lg_n - 1 - lg_hlo - l));
    };
    constexpr int NPAIR = K / 2;
#pragma unroll 1
    for (int pr = 0; pr < NPAIR; pr++) {
        // DIF: levels (hi, hi - 1) from K - 1 down; DIT: (lo, lo + 1) from 0 up
        const int l = DIT ? 2 * pr : K - 1 - 2 * pr;
        const int lb = DIT ? l : l - 1;
        const int step = 2 * pr;  // the pass's step of the pair's first level (k_ntt_pass29 numbering)
        for (int q = threadIdx.x; q < TILE / 4; q += NTT4_THREADS) {
            const int g = q % G, q4 = q / G;
            const uint32_t ml = q4 & ((1 << lb) - 1);
            const int m = ((q4 >> lb) << (lb + 2)) | (int)ml;
            const int e0 = m * G + g, e1 = (m + (1 << lb)) * G + g, e2 = (m + (2 << lb)) * G + g,
                      e3 = (m + (3 << lb)) * G + g;
            const uint64_t j = (gid0 + g) & (hlo - 1);
            R29 x0 = get(e0), x1 = get(e1), x2 = get(e2), x3 = get(e3);
            const bool unit = lg_hlo == 0 && lb == 0;  // level lb has half size 1
            if (DIT) {
                // level lb (step): (x0, x1), (x2, x3), one twiddle
                R29 t0 = x1, t1 = x3;
                if (!unit) {
                    const R29 w = twl(j, lb, ml);
                    t0 = r29_mul(x1, w);
                    t1 = r29_mul(x3, w);
                }
                x1 = r29_sub(x0, t0, R29_KDIT); x0 = r29_add(x0, t0);
                x3 = r29_sub(x2, t1, R29_KDIT); x2 = r29_add(x2, t1);
                // level lb + 1 (step + 1): (x0, x2) low bits ml, (x1, x3) ml + 2^lb
                R29 t = r29_mul(x2, twl(j, lb + 1, ml));
                x2 = r29_sub(x0, t, R29_KDIT); x0 = r29_add(x0, t);
                t = r29_mul(x3, twl(j, lb + 1, ml + (1u << lb)));
                x3 = r29_sub(x1, t, R29_KDIT); x1 = r29_add(x1, t);
            } else {
                // level lb + 1 (step): (x0, x2) low bits ml, (x1, x3) ml + 2^lb
                const uint32_t *k0 = R29_KDIF[step], *k1 = R29_KDIF[step + 1];
                R29 d = r29_mul(r29_sub(x0, x2, k0), twl(j, lb + 1, ml)); x0 = r29_add(x0, x2); x2 = d;
                d = r29_mul(r29_sub(x1, x3, k0), twl(j, lb + 1, ml + (1u << lb))); x1 = r29_add(x1, x3); x3 = d;
                // level lb (step + 1): (x0, x1), (x2, x3)
                if (unit) {
                    d = r29_sub(x0, x1, k1); x0 = r29_add(x0, x1); x1 = d;
                    d = r29_sub(x2, x3, k1); x2 = r29_add(x2, x3); x3 = d;
                } else {
                    const R29 w = twl(j, lb, ml);
                    d = r29_mul(r29_sub(x0, x1, k1), w); x0 = r29_add(x0, x1); x1 = d;
                    d = r29_mul(r29_sub(x2, x3, k1), w); x2 = r29_add(x2, x3); x3 = d;
                }
            }
            put(e0, x0);
            put(e1, x1);
            put(e2, x2);
            put(e3, x3);
        }
        __syncthreads();
    }
    if (K & 1) {  // the remaining level: DIF level 0 (step K - 1), DIT level K - 1
        const int l = DIT ? K - 1 : 0;
        const bool unit = lg_hlo == 0 && l == 0;
        const uint32_t *kd = R29_KDIF[K - 1];
        for (int bf = threadIdx.x; bf < TILE / 2; bf += NTT4_THREADS) {
            const int g = bf % G, q = bf / G;
            const int mlow = q & ((1 << l) - 1);
            const int m = ((q >> l) << (l + 1)) | mlow;
            const int e0 = m * G + g, e1 = (m + (1 << l)) * G + g;
            const uint64_t j = (gid0 + g) & (hlo - 1);
            const R29 a = get(e0), b = get(e1);
            R29 s2, d;
            if (DIT) {
                const R29 t = unit ? b : r29_mul(b, twl(j, l, (uint32_t)mlow));
                s2 = r29_add(a, t);
                d = r29_sub(a, t, R29_KDIT);
            } else {
                s2 = r29_add(a, b);
                d = r29_sub(a, b, kd);
                if (!unit) d = r29_mul(d, twl(j, l, (uint32_t)mlow));
            }
            put(e0, s2);
            put(e1, d);
        }
        __syncthreads();
    }
    for (int e = threadIdx.x; e < TILE; e += NTT4_THREADS) {
        const int g = e % G, m = e / G;
        const uint64_t gid = gid0 + g;
        const uint64_t j = gid & (hlo - 1), b = gid >> lg_hlo;
        const uint64_t idx = (b << (lg_hlo + K)) + j + ((uint64_t)m << lg_hlo);
        R29 x = get(e);
        if (post) x = r29_mul(x, r29_load(post, idx));
        x = r29_canon(x);
        uint32_t w[8];
        r29_to_words(x, w);
        uint4 *dst = reinterpret_cast<uint4 *>(data + 4 * idx);
        dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
        dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
    }
}

// small transforms (N < TILE): one workgroup does everything in LDS
template <bool DIT>
__global__ __launch_bounds__(NTT_THREADS) void k_ntt_small(uint64_t *data, const uint64_t *tw,
                                                            uint32_t lg_n) {
    __shared__ uint4 lds_lo[TILE];
    __shared__ uint4 lds_hi[TILE];
    const int n = 1 << lg_n;
    for (int e = threadIdx.x; e < n; e += NTT_THREADS) {
        const uint4 *src = reinterpret_cast<const uint4 *>(data + 4 * (uint64_t)e);
        lds_lo[e] = src[0];
        lds_hi[e] = src[1];
    }
    __syncthreads();
    for (int step = 0; step < (int)lg_n; step++) {
        const int l = DIT ? step : (int)lg_n - 1 - step;
        for (int bf = threadIdx.x; bf < n / 2; bf += NTT_THREADS) {
            int mlow = bf & ((1 << l) - 1);
            int m = ((bf >> l) << (l + 1)) | mlow;
            int e0 = m, e1 = m + (1 << l);
            Fr w = load_fr(tw, (uint64_t)mlow << (lg_n - 1 - l));
            uint4 a0 = lds_lo[e0], a1 = lds_hi[e0], b0 = lds_lo[e1], b1 = lds_hi[e1];
            Fr a, b;
            a.v[0] = a0.x; a.v[1] = a0.y; a.v[2] = a0.z; a.v[3] = a0.w;
            a.v[4] = a1.x; a.v[5] = a1.y; a.v[6] = a1.z; a.v[7] = a1.w;
            b.v[0] = b0.x; b.v[1] = b0.y; b.v[2] = b0.z; b.v[3] = b0.w;
            b.v[4] = b1.x; b.v[5] = b1.y; b.v[6] = b1.z; b.v[7] = b1.w;
            Fr s, d;
            if (DIT) {
                Fr t = b * w;
                s = a + t;
                d = a - t;
            } else {
                s = a + b;
                d = (a - b) * w;
            }
            lds_lo[e0] = make_uint4(s.v[0], s.v[1], s.v[2], s.v[3]);
            lds_hi[e0] = make_uint4(s.v[4], s.v[5], s.v[6], s.v[7]);
            lds_lo[e1] = make_uint4(d.v[0], d.v[1], d.v[2], d.v[3]);
            lds_hi[e1] = make_uint4(d.v[4], d.v[5], d.v[6], d.v[7]);
        }
        __syncthreads();
    }
    for (int e = threadIdx.x; e < n; e += NTT_THREADS) {
        uint4 *dst = reinterpret_cast<uint4 *>(data + 4 * (uint64_t)e);
        dst[0] = lds_lo[e];
        dst[1] = lds_hi[e];
    }
}

// ---------------------------------------------------------------- bit reversal
__device__ __forceinline__ uint32_t brev(uint32_t x, uint32_t bits) {
    return __brev(x) >> (32 - bits);
}

// mode 0: plain, 1: * c, 2: * c * g^-i (i = natural output index)
struct Scale {
    int mode;
    Fr c;
    const uint64_t *hi, *lo;
};
__device__ __forceinline__ Fr apply_scale(const Scale &s, Fr x, uint64_t i) {
    if (s.mode == 0) return x;
    Fr f = s.c;
    if (s.mode == 2) f = f * coset_pow(s.hi, s.lo, i);
    return x * f;
}

// lg >= 2 TB: index = hi | mid | lo (TB bits each end); tile(mid) <->
// tile(rev(mid)) transposed.  TB = 4 (default): 16 x 16 tiles, 17 KB of LDS
// per workgroup, one element per lane per tile; TB = 5 (32 x 32, 68 KB: two
// workgroups per CU) moved 256 MB in ~0.3 ms at 2^22, ~0.9 TB/s.  Rows of a
// tile are 2^TB consecutive elements (512 B at TB = 4: four whole lines).
template <int TB>
__global__ __launch_bounds__(256) void k_bitrev_tiles(uint64_t *data, uint32_t lg, Scale sc) {
    constexpr int T = 1 << TB, TP = T + 1;
    __shared__ uint4 t0l[T * TP], t0h[T * TP], t1l[T * TP], t1h[T * TP];
    data += ((uint64_t)blockIdx.y << lg) * 4;  // independent transforms of 2^lg side by side
    const uint32_t midbits = lg - 2 * TB;
    const uint32_t mid = blockIdx.x;
    const uint32_t rmid = midbits ? brev(mid, midbits) : 0;
    if (rmid < mid) return;  // each pair handled once
    const bool self = rmid == mid;
    // load tile(mid): rows hi, cols lo contiguous
    for (int e = threadIdx.x; e < T * T; e += 256) {
        uint32_t h = e >> TB, l = e & (T - 1);
        uint64_t i0 = ((uint64_t)h << (lg - TB)) | ((uint64_t)mid << TB) | l;
        const uint4 *s0 = reinterpret_cast<const uint4 *>(data + 4 * i0);
        t0l[h * TP + l] = s0[0];
        t0h[h * TP + l] = s0[1];
        if (!self) {
            uint64_t i1 = ((uint64_t)h << (lg - TB)) | ((uint64_t)rmid << TB) | l;
            const uint4 *s1 = reinterpret_cast<const uint4 *>(data + 4 * i1);
            t1l[h * TP + l] = s1[0];
            t1h[h * TP + l] = s1[1];
        }
    }
    __syncthreads();
    // element at (h, mid, l) goes to (rev(l), rev(mid), rev(h)).
    // write tile position rmid: dest (h', rmid, l') gets source (rev(l'), mid, rev(h'))
    for (int e = threadIdx.x; e < T * T; e += 256) {
        uint32_t h2 = e >> TB, l2 = e & (T - 1);
        uint32_t sh = brev(l2, TB), sl = brev(h2, TB);
        uint64_t d0 = ((uint64_t)h2 << (lg - TB)) | ((uint64_t)rmid << TB) | l2;
        Fr x;
        uint4 lo = t0l[sh * TP + sl], hi = t0h[sh * TP + sl];
        x.v[0] = lo.x; x.v[1] = lo.y; x.v[2] = lo.z; x.v[3] = lo.w;
        x.v[4] = hi.x; x.v[5] = hi.y; x.v[6] = hi.z; x.v[7] = hi.w;
        store_fr(data, d0, apply_scale(sc, x, d0));
        if (!self) {
            uint64_t d1 = ((uint64_t)h2 << (lg - TB)) | ((uint64_t)mid << TB) | l2;
            uint4 lo1 = t1l[sh * TP + sl], hi1 = t1h[sh * TP + sl];
            Fr y;
            y.v[0] = lo1.x; y.v[1] = lo1.y; y.v[2] = lo1.z; y.v[3] = lo1.w;
            y.v[4] = hi1.x; y.v[5] = hi1.y; y.v[6] = hi1.z; y.v[7] = hi1.w;
            store_fr(data, d1, apply_scale(sc, y, d1));
        }
    }
}

// lg < 10: single workgroup, via LDS
__global__ __launch_bounds__(256) void k_bitrev_small(uint64_t *data, uint32_t lg, Scale sc) {
    __shared__ uint4 tl[1024], th[1024];
    data += ((uint64_t)blockIdx.y << lg) * 4;
    const uint32_t n = 1u << lg;
    for (uint32_t e = threadIdx.x; e < n; e += 256) {
        const uint4 *s = reinterpret_cast<const uint4 *>(data + 4 * (uint64_t)e);
        tl[e] = s[0];
        th[e] = s[1];
    }
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < n; e += 256) {
        uint32_t src = lg ? brev(e, lg) : 0;
        Fr x;
        uint4 lo = tl[src], hi = th[src];
        x.v[0] = lo.x; x.v[1] = lo.y; x.v[2] = lo.z; x.v[3] = lo.w;
        x.v[4] = hi.x; x.v[5] = hi.y; x.v[6] = hi.z; x.v[7] = hi.w;
        store_fr(data, e, apply_scale(sc, x, e));
    }
}

// forward coset: x_i *= g^i
__global__ void k_coset_scale(uint64_t *data, uint64_t n, const uint64_t *hi, const uint64_t *lo) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    store_fr(data, i, load_fr(data, i) * coset_pow(hi, lo, i));
}

// out[i] = i < n ? in[i] * g^i : 0   (pad_poly + LDE_distribute_powers)
__global__ void k_pad_coset(const uint64_t *in, uint64_t *out, uint64_t n, uint64_t N,
                            const uint64_t *hi, const uint64_t *lo) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= N) return;
    Fr x = Fr::zero();
    if (i < n) x = load_fr(in, i) * coset_pow(hi, lo, i);
    store_fr(out, i, x);
}

// Fused extras of the first (src, pre) and last (post) pass, see k_ntt_pass
struct PassFuse {
    const uint64_t *src = nullptr, *pre = nullptr, *post = nullptr;
    uint64_t src_mask = 0;
    const uint32_t *pre29 = nullptr, *post29 = nullptr;  // the 2^261 forms of pre / post
};

// PNP_NTT_R4=0: the radix-2 passes (k_ntt_pass) instead of k_ntt_pass4
static bool ntt4_enabled() {
    static const bool on = [] {
        const char *e = getenv("PNP_NTT_R4");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

// PNP_NTT29=1: the radix-2^29 passes (k_ntt_pass29).  Measured SLOWER than the
// 32-bit-limb passes on MI355X (same-box, n = 2^22: 12.9 vs 11.6 ms for the
// <7, DIF> passes of a proof): the v_addc_co_u32 of the 32-bit product issues
// at the full VALU rate inside the multiply-add chain, so the 29-bit product
// saves fewer cycles than its 36-byte LDS planes (4 instead of 5 workgroups
// per CU), extra LDS instructions and per-pass canonicalisation cost.
static bool ntt29_enabled() {
    static const bool on = [] {
        const char *e = getenv("PNP_NTT29");
        return e && atoi(e) != 0;
    }();
    return on;
}
__global__ void k_mul_table(uint64_t *d, const uint64_t *T, uint64_t N);
__global__ void k_lde_twist(const uint64_t *in, const uint64_t *T, uint64_t *out, uint64_t n, uint64_t N);

// DIF (natural -> bit-reversed) or DIT (bit-reversed -> natural) of size 2^lg
// on each of `count` consecutive blocks of 2^lg elements (any count: the
// round-4 coset blocks number 6 or 8)
static void ntt_core(NttTables &t, uint64_t *d, uint32_t lg, bool inverse, bool dit, hipStream_t s,
                     uint64_t count = 1, const PassFuse &fz = PassFuse()) {
    const uint64_t N = count << lg;
    const uint64_t *tw = ntt_twiddles(t, lg, inverse, s);
    // LDS-tile passes need whole tiles (a tile holds TILE >> lg transforms when
    // lg < LGTILE); otherwise one single-workgroup transform per block
    if (N % TILE != 0 || (lg <= (uint32_t)LGTILE && count == 1)) {
        if (fz.src && fz.pre) {
            hipLaunchKernelGGL(k_lde_twist, dim3((uint32_t)((N + 255) / 256)), dim3(256), 0, s, fz.src,
                               fz.pre, d, fz.src_mask + 1, N);
            PNP_HIP(hipGetLastError());
        } else if (fz.src) {  // out of place, no twist (src_mask covers N)
            PNP_HIP(hipMemcpyAsync(d, fz.src, 32 * N, hipMemcpyDeviceToDevice, s));
        }
        for (uint64_t b = 0; b < count; b++) {
            if (dit)
                hipLaunchKernelGGL(k_ntt_small<true>, dim3(1), dim3(NTT_THREADS), 0, s, d + 4 * (b << lg), tw, lg);
            else
                hipLaunchKernelGGL(k_ntt_small<false>, dim3(1), dim3(NTT_THREADS), 0, s, d + 4 * (b << lg), tw, lg);
            PNP_HIP(hipGetLastError());
        }
        if (fz.post) {
            hipLaunchKernelGGL(k_mul_table, dim3((uint32_t)((N + 255) / 256)), dim3(256), 0, s, d, fz.post, N);
            PNP_HIP(hipGetLastError());
        }
        return;
    }
    // split lg into passes of at most LGTILE levels (balanced); DIF runs them from
    // the largest half size down, DIT from the smallest up
    const int npass = (lg + LGTILE - 1) / LGTILE;
    int ks[4], rem = lg;
    for (int p = 0; p < npass; p++) {
        ks[p] = (rem + (npass - p) - 1) / (npass - p);
        rem -= ks[p];
    }
    uint32_t lo = dit ? 0 : lg;  // DIF: current top exponent; DIT: current bottom
    // radix 2^29 (PNP_NTT29): every pass of at most 8 levels (R29_KDIF's
    // steps), with the 2^261-form twists where a pass fuses one
    bool r29 = ntt29_enabled() && (!fz.pre || fz.pre29) && (!fz.post || fz.post29);
    for (int p = 0; p < npass; p++) r29 &= ks[p] <= 8;
    const uint32_t *tw29 = r29 ? ntt_twiddles29(t, lg, inverse, s) : nullptr;
    for (int p = 0; p < npass; p++) {
        const int k = ks[p];
        const uint32_t lg_hlo = dit ? lo : lo - k;
        const uint32_t blocks = (uint32_t)((N >> k) / (TILE >> k));
        const uint64_t *src = p == 0 ? fz.src : nullptr, *pre = p == 0 ? fz.pre : nullptr;
        const uint64_t *post = p == npass - 1 ? fz.post : nullptr;
        if (r29 && k >= 2 && ntt4_enabled()) {
            const uint32_t *pre29 = p == 0 ? fz.pre29 : nullptr, *post29 = p == npass - 1 ? fz.post29 : nullptr;
            const uint32_t b4 = (uint32_t)((N >> k) / (TILE >> k));
            switch (k) {
#define PNP_CASE429(KK)                                                                                 \
    case KK:                                                                                            \
        if (dit)                                                                                        \
            hipLaunchKernelGGL((k_ntt_pass4_29<KK, true>), dim3(b4), dim3(NTT4_THREADS), 0, s, d, tw29, \
                               lg, lg_hlo, src, pre29, fz.src_mask, post29);                           \
        else                                                                                            \
            hipLaunchKernelGGL((k_ntt_pass4_29<KK, false>), dim3(b4), dim3(NTT4_THREADS), 0, s, d, tw29, \
                               lg, lg_hlo, src, pre29, fz.src_mask, post29);                           \
        break;
                PNP_CASE429(2) PNP_CASE429(3) PNP_CASE429(4) PNP_CASE429(5)
                PNP_CASE429(6) PNP_CASE429(7) PNP_CASE429(8)
#undef PNP_CASE429
            }
            PNP_HIP(hipGetLastError());
            lo = dit ? lo + k : lo - k;
            continue;
        }
        if (r29 && (!src || pre)) {
            const uint32_t *pre29 = p == 0 ? fz.pre29 : nullptr, *post29 = p == npass - 1 ? fz.post29 : nullptr;
            switch (k) {
#define PNP_CASE29(KK)                                                                              \
    case KK:                                                                                        \
        if (dit)                                                                                    \
            hipLaunchKernelGGL((k_ntt_pass29<KK, true>), dim3(blocks), dim3(NTT_THREADS), 0, s, d, tw29, \
                               lg, lg_hlo, src, pre29, fz.src_mask, post29);                       \
        else                                                                                        \
            hipLaunchKernelGGL((k_ntt_pass29<KK, false>), dim3(blocks), dim3(NTT_THREADS), 0, s, d, tw29, \
                               lg, lg_hlo, src, pre29, fz.src_mask, post29);                       \
        break;
                PNP_CASE29(1) PNP_CASE29(2) PNP_CASE29(3) PNP_CASE29(4)
                PNP_CASE29(5) PNP_CASE29(6) PNP_CASE29(7) PNP_CASE29(8)
#undef PNP_CASE29
            }
            PNP_HIP(hipGetLastError());
            lo = dit ? lo + k : lo - k;
            continue;
        }
        if (ntt4_enabled() && k >= 2) {
            const int rows = ntt_rows_enabled() ? 1 : 0;
            const uint64_t *tw4 = rows ? ntt_twiddle_rows(t, lg, inverse, s) : tw;
            switch (k) {
#define PNP_CASE4(KK)                                                                               \
    case KK:                                                                                        \
        if (dit)                                                                                    \
            hipLaunchKernelGGL((k_ntt_pass4<KK, true>), dim3(blocks), dim3(NTT4_THREADS), 0, s, d, tw4, \
                               lg, lg_hlo, src, pre, fz.src_mask, post, rows);                     \
        else                                                                                        \
            hipLaunchKernelGGL((k_ntt_pass4<KK, false>), dim3(blocks), dim3(NTT4_THREADS), 0, s, d, tw4, \
                               lg, lg_hlo, src, pre, fz.src_mask, post, rows);                     \
        break;
                PNP_CASE4(2) PNP_CASE4(3) PNP_CASE4(4) PNP_CASE4(5) PNP_CASE4(6)
                PNP_CASE4(7) PNP_CASE4(8) PNP_CASE4(9) PNP_CASE4(10)
#if PNP_NTT_LGTILE >= 11
                PNP_CASE4(11)
#endif
#undef PNP_CASE4
                default:
                    set_error("bad NTT pass size %d", k);
                    throw Error(PNP_E_ARG);
            }
            PNP_HIP(hipGetLastError());
            lo = dit ? lo + k : lo - k;
            continue;
        }
        switch (k) {
#define PNP_CASE(KK)                                                                               \
    case KK:                                                                                       \
        if (dit)                                                                                   \
            hipLaunchKernelGGL((k_ntt_pass<KK, true>), dim3(blocks), dim3(NTT_THREADS), 0, s, d, tw, \
                               lg, lg_hlo, src, pre, fz.src_mask, post);                          \
        else                                                                                       \
            hipLaunchKernelGGL((k_ntt_pass<KK, false>), dim3(blocks), dim3(NTT_THREADS), 0, s, d, tw, \
                               lg, lg_hlo, src, pre, fz.src_mask, post);                          \
        break;
            PNP_CASE(1) PNP_CASE(2) PNP_CASE(3) PNP_CASE(4) PNP_CASE(5)
            PNP_CASE(6) PNP_CASE(7) PNP_CASE(8) PNP_CASE(9) PNP_CASE(10)
#if PNP_NTT_LGTILE >= 11
            PNP_CASE(11)
#endif
#undef PNP_CASE
            default:
                set_error("bad NTT pass size %d", k);
                throw Error(PNP_E_ARG);
        }
        PNP_HIP(hipGetLastError());
        lo = dit ? lo + k : lo - k;
    }
}

static void dif(NttTables &t, uint64_t *d, uint32_t lg, bool inverse, hipStream_t s, uint64_t count = 1) {
    ntt_core(t, d, lg, inverse, false, s, count);
}

static void bitrev(uint64_t *d, uint32_t lg, const Scale &sc, hipStream_t s, uint32_t nblocks = 1) {
    static const int tb = getenv("PNP_BITREV_TB") && atoi(getenv("PNP_BITREV_TB")) == 5 ? 5 : 4;  // A/B
    if (lg < 10) {
        hipLaunchKernelGGL(k_bitrev_small, dim3(1, nblocks), dim3(256), 0, s, d, lg, sc);
    } else if (tb == 5) {
        hipLaunchKernelGGL(k_bitrev_tiles<5>, dim3(1u << (lg - 10), nblocks), dim3(256), 0, s, d, lg, sc);
    } else {
        hipLaunchKernelGGL(k_bitrev_tiles<4>, dim3(1u << (lg - 8), nblocks), dim3(256), 0, s, d, lg, sc);
    }
    PNP_HIP(hipGetLastError());
}

void ntt_run(NttTables &t, uint64_t *d, uint32_t lg, bool inverse, bool coset, hipStream_t s,
             const uint64_t *src) {
    uint64_t n = 1ULL << lg;
    if (src && src != d && (lg == 0 || (!inverse && coset))) {
        PNP_HIP(hipMemcpyAsync(d, src, 32 * n, hipMemcpyDeviceToDevice, s));
        src = nullptr;
    }
    if (lg == 0) return;
    if (coset) ntt_prepare_coset(t, s);
    if (!inverse && coset) {
        hipLaunchKernelGGL(k_coset_scale, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, d, n,
                           t.coset_hi.u64(), t.coset_lo.u64());
        PNP_HIP(hipGetLastError());
    }
    if (src && src != d) {  // the first pass reads src: no separate copy
        PassFuse fz;
        fz.src = src;
        fz.src_mask = n - 1;
        ntt_core(t, d, lg, inverse, false, s, 1, fz);
    } else {
        dif(t, d, lg, inverse, s);
    }
    Scale sc{0, Fr::one(), nullptr, nullptr};
    if (inverse) {
        Fr nf = Fr::zero();
        nf.v[0] = (uint32_t)n;
        nf.v[1] = (uint32_t)(n >> 32);
        sc.mode = coset ? 2 : 1;
        sc.c = pnp::inverse(to_mont(nf));
        sc.hi = t.coset_inv_hi.u64();
        sc.lo = t.coset_inv_lo.u64();
    }
    bitrev(d, lg, sc, s);
}

// out[b n + j] = in[j] * T[b n + j],  T[b n + j] = (g w_8n^rev3(b))^j
__global__ void k_lde_twist(const uint64_t *in, const uint64_t *T, uint64_t *out, uint64_t n,
                            uint64_t N) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= N) return;
    store_fr(out, i, load_fr(in, i & (n - 1)) * load_fr(T, i));
}

static const uint64_t *lde_twist_table(NttTables &t, uint32_t lg_n, hipStream_t s) {
    auto it = t.lde_twist.find(lg_n);
    if (it != t.lde_twist.end()) return it->second.u64();
    const uint64_t n = 1ULL << lg_n;
    DevBuf buf(8 * n * 32);
    const Fr w8n = host_root(lg_n + 3), g = host_gen();
    const uint32_t chunk = 64;
    const uint64_t threads = (n + chunk - 1) / chunk;
    for (uint32_t b = 0; b < 8; b++) {
        uint32_t m = ((b & 1) << 2) | (b & 2) | ((b >> 2) & 1);  // rev3(b)
        Fr base = g * pow_u64(w8n, m);
        hipLaunchKernelGGL(k_powers_table, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, s,
                           buf.u64() + 4 * b * n, n, base, chunk);
        PNP_HIP(hipGetLastError());
    }
    const uint64_t *p = buf.u64();
    t.lde_twist.emplace(lg_n, std::move(buf));
    return p;
}

// Ntt_coset::forward of the zero-padded n-coefficient polynomial on 8n points.
// The top three DIF levels of a length-8n transform whose upper 7n inputs are
// zero only copy and twist: afterwards block b (of 8, length n) holds
// c_j g^j w_8n^(j rev3(b)).  So: one twist pass from a key-independent table,
// then 22 (not 25) DIF levels as 8 independent size-n transforms (their
// twiddle table is 8x smaller and stays in the MALL), then the usual 8n
// bit reversal to natural order.
void coset_lde8(NttTables &t, const uint64_t *in, uint64_t *out8, uint32_t lg_n, hipStream_t s) {
    uint64_t n = 1ULL << lg_n, N = n << 3;
    const uint64_t *T = lde_twist_table(t, lg_n, s);
    hipLaunchKernelGGL(k_lde_twist, dim3((uint32_t)((N + 255) / 256)), dim3(256), 0, s, in, T, out8,
                       n, N);
    PNP_HIP(hipGetLastError());
    if (lg_n > 0) dif(t, out8, lg_n, false, s, 8);
    Scale sc{0, Fr::one(), nullptr, nullptr};
    bitrev(out8, lg_n + 3, sc, s);
}

// ---------------------------------------------------------------- block layout
// gen_proof round 4 keeps the 8n coset in "block layout": point
// x_i = g w_8n^i, i = 8 j + m, lives in block m at index j, so each residue
// class m is the size-n domain coset g w_8n^m <w_n> and every block is an
// independent size-n transform (and a unit of multi-GPU work).
static const uint64_t *block_twist_table(NttTables &t, uint32_t lg_n, bool inverse, hipStream_t s) {
    auto &tabs = inverse ? t.blk_twist_inv : t.blk_twist;
    auto it = tabs.find(lg_n);
    if (it != tabs.end()) return it->second.u64();
    const uint64_t n = 1ULL << lg_n;
    DevBuf buf(8 * n * 32);
    const Fr w8n = host_root(lg_n + 3), g = host_gen();
    const uint32_t chunk = 64;
    const uint64_t threads = (n + chunk - 1) / chunk;
    for (uint32_t m = 0; m < 8; m++) {
        // forward: (g w_8n^m)^j;  inverse: w_8n^(-m j)
        Fr base = inverse ? pnp::inverse(pow_u64(w8n, m)) : g * pow_u64(w8n, m);
        hipLaunchKernelGGL(k_powers_table, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, s,
                           buf.u64() + 4 * m * n, n, base, chunk);
        PNP_HIP(hipGetLastError());
    }
    const uint64_t *p = buf.u64();
    tabs.emplace(lg_n, std::move(buf));
    return p;
}

// the forward block twists times 32: an LDE through them yields 32 f(x) in
// the 2^256 form, i.e. f(x) in the 2^261 form of fr29.cuh (k_quotient29's
// inputs, protocol.hip), at no cost in the transform
__global__ void k_times32(const uint64_t *in, uint64_t *out, uint64_t N) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= N) return;
    Fr x = load_fr(in, i);
#pragma unroll
    for (int k = 0; k < 5; k++) x = x + x;
    store_fr(out, i, x);
}
static const uint64_t *block_twist_table32(NttTables &t, uint32_t lg_n, hipStream_t s) {
    auto it = t.blk_twist32.find(lg_n);
    if (it != t.blk_twist32.end()) return it->second.u64();
    const uint64_t N = 8ULL << lg_n;
    const uint64_t *src = block_twist_table(t, lg_n, false, s);
    DevBuf buf(N * 32);
    hipLaunchKernelGGL(k_times32, dim3((uint32_t)((N + 255) / 256)), dim3(256), 0, s, src, buf.u64(), N);
    PNP_HIP(hipGetLastError());
    const uint64_t *p = buf.u64();
    t.blk_twist32.emplace(lg_n, std::move(buf));
    return p;
}

static void check_blocks(int m0, int nb) {
    if (m0 < 0 || nb < 1 || m0 + nb > 8) {
        set_error("coset blocks [%d, %d) outside [0, 8)", m0, m0 + nb);
        throw Error(PNP_E_ARG);
    }
}

// out[b n + brev(j)] = f(g w_8n^(8 j + m0 + b)), b < nb, for the n
// coefficients `in`: the twist is fused into the first DIF pass and the DIF's
// bit-reversed output is kept ("block-bitrev layout", no reversal pass); the
// quotient's arrays share the layout and intt_blocks undoes it with a DIT.
static const uint32_t *block_twist_table29(NttTables &t, uint32_t lg_n, bool inverse, hipStream_t s) {
    return to_r29_table(inverse ? t.blk_twist_inv29 : t.blk_twist29, lg_n, block_twist_table(t, lg_n, inverse, s),
                        8ULL << lg_n, s);
}
// the forward twists times 32 in the 2^261 form (the radix-2^29 LDE into k_quotient29's form)
static const uint32_t *block_twist_table32_29(NttTables &t, uint32_t lg_n, hipStream_t s) {
    return to_r29_table(t.blk_twist32_29, lg_n, block_twist_table32(t, lg_n, s), 8ULL << lg_n, s);
}

// Every table a proof of domain 2^lg_n reads, built on stream s.  The tables
// are otherwise built lazily by their first user; a proof forks LDEs onto a
// side stream, so prove_impl builds them on its main stream before the first
// fork (the side stream then waits for them through the fork event).
void ntt_warm(NttTables &t, uint32_t lg_n, hipStream_t s) {
    for (bool inv : {false, true}) {
        ntt_twiddles(t, lg_n, inv, s);
        block_twist_table(t, lg_n, inv, s);
        if (ntt29_enabled()) {
            ntt_twiddles29(t, lg_n, inv, s);
            block_twist_table29(t, lg_n, inv, s);
        }
    }
    block_twist_table32(t, lg_n, s);
    if (ntt29_enabled()) block_twist_table32_29(t, lg_n, s);
    ntt_prepare_coset(t, s);
}

void lde_blocks(NttTables &t, const uint64_t *in, uint64_t *out, uint32_t lg_n, int m0, int nb,
                hipStream_t s, bool form29) {
    const uint64_t n = 1ULL << lg_n;
    PassFuse fz;
    fz.src = in;
    // (form29: the 32-bit passes; the experimental radix-2^29 passes have no scaled twist)
    fz.pre = (form29 ? block_twist_table32(t, lg_n, s) : block_twist_table(t, lg_n, false, s)) + 4 * (uint64_t)m0 * n;
    if (ntt29_enabled())
        fz.pre29 = (form29 ? block_twist_table32_29(t, lg_n, s) : block_twist_table29(t, lg_n, false, s)) +
                   9 * (uint64_t)m0 * n;
    fz.src_mask = n - 1;
    check_blocks(m0, nb);
    ntt_core(t, out, lg_n, false, false, s, (uint64_t)nb, fz);
}

__global__ void k_mul_table(uint64_t *d, const uint64_t *T, uint64_t N) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < N) store_fr(d, i, load_fr(d, i) * load_fr(T, i));
}

// in place, block b < nb holding residue m = m0 + b in block-bitrev layout:
//   Y_m[u] = w_8n^(-m u) sum_j d[b n + brev(j)] w_n^(-j u)      (no 1/n scaling)
// as a DIT (bit-reversed in, natural out) with the twist fused into its last pass
void intt_blocks(NttTables &t, uint64_t *d, uint32_t lg_n, int m0, int nb, hipStream_t s) {
    const uint64_t n = 1ULL << lg_n;
    PassFuse fz;
    fz.post = block_twist_table(t, lg_n, true, s) + 4 * (uint64_t)m0 * n;
    if (ntt29_enabled()) fz.post29 = block_twist_table29(t, lg_n, true, s) + 9 * (uint64_t)m0 * n;
    check_blocks(m0, nb);
    ntt_core(t, d, lg_n, true, true, s, (uint64_t)nb, fz);
}

// Coefficients of the 8n-point coset interpolant from the 8 twisted block
// transforms Y_m (block-major, `len` entries each, covering u in [q0, q0+len)):
//   c_(u + n m1) = g^-(u + n m1) / (8n) sum_m w_8^(-m m1) Y_m[u]
// -> out[m1 len + (u - q0)]: radix-2 8-point inverse DFT per u.
// M < 8 blocks (deg t < M n, prover.cpp): the chunks m1 >= M are zero, i.e.
// sum_m w_8^(-m m1) Y_m = 0 for m1 = M .. 7 — 8 - M linear equations that give
// the missing Y_M .. Y_7 from Y_0 .. Y_(M-1) (ext, solved on the host); then
// the same inverse DFT, and only the chunks m1 < M are stored.
template <int M>
struct TcombExt {
    Fr c[M < 8 ? (8 - M) * M : 1];
};
// nz: bit m1 set when chunk m1 has a non-zero coefficient in this range (the
// chunks that are zero commit to infinity without an MSM)
template <int M>
__global__ __launch_bounds__(256) void k_t_combine(const uint64_t *Y, uint64_t len, uint64_t q0, uint64_t *out,
                                                   TcombExt<M> ext, Fr w1, Fr w2, Fr w3, Fr inv8n,
                                                   const uint64_t *chi, const uint64_t *clo, Fr gn0, Fr gn1,
                                                   Fr gn2, Fr gn3, Fr gn4, Fr gn5, Fr gn6, Fr gn7,
                                                   unsigned *nz) {
    __shared__ unsigned bm;
    if (threadIdx.x == 0) bm = 0;
    __syncthreads();
    const uint64_t u = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (u < len) {
    Fr y[8];
#pragma unroll
    for (int m = 0; m < M; m++) y[m] = load_fr(Y, m * len + u);
#pragma unroll
    for (int e = 0; e < 8 - M; e++) {
        // products in pairs sharing one Montgomery reduction (fr_mul2)
        Fr acc = M % 2 ? ext.c[e * M + M - 1] * y[M - 1] : Fr::zero();
#pragma unroll
        for (int m = 0; m + 1 < M; m += 2) acc += fr_mul2(ext.c[e * M + m], y[m], ext.c[e * M + m + 1], y[m + 1]);
        y[M + e] = acc;
    }
    // DIF stage h = 4 (twiddles w^k), h = 2 (w^2k), h = 1; output bit-reversed
    const Fr wk[4] = {Fr::one(), w1, w2, w3};
#pragma unroll
    for (int k = 0; k < 4; k++) {
        Fr a = y[k], b = y[k + 4];
        y[k] = a + b;
        y[k + 4] = k ? (a - b) * wk[k] : a - b;
    }
#pragma unroll
    for (int base = 0; base < 8; base += 4) {
        Fr a = y[base], b = y[base + 2];
        y[base] = a + b;
        y[base + 2] = a - b;
        a = y[base + 1];
        b = y[base + 3];
        y[base + 1] = a + b;
        y[base + 3] = (a - b) * w2;
    }
#pragma unroll
    for (int base = 0; base < 8; base += 2) {
        Fr a = y[base], b = y[base + 1];
        y[base] = a + b;
        y[base + 1] = a - b;
    }
    const Fr s0 = coset_pow(chi, clo, q0 + u) * inv8n;  // g^-u / (8n)
    const Fr gn[8] = {gn0, gn1, gn2, gn3, gn4, gn5, gn6, gn7};
    const int rev[8] = {0, 4, 2, 6, 1, 5, 3, 7};
    unsigned mask = 0;
#pragma unroll
    for (int p = 0; p < 8; p++) {
        const int m1 = rev[p];
        if (m1 < M) {
            const Fr v = y[p] * (s0 * gn[m1]);
            store_fr(out, m1 * len + u, v);
            if (!v.is_zero()) mask |= 1u << m1;
        }
    }
    if (mask) atomicOr(&bm, mask);
    }
    __syncthreads();
    if (threadIdx.x == 0 && bm) atomicOr(nz, bm);
}

template <int M>
static void t_combine_m(NttTables &t, const uint64_t *Y, uint64_t len, uint64_t q0, uint64_t *out,
                        uint32_t lg_n, unsigned *nz, hipStream_t s) {
    ntt_prepare_coset(t, s);
    const uint64_t n = 1ULL << lg_n;
    const Fr w8i = pnp::inverse(host_root(3));
    Fr w[4] = {Fr::one(), w8i, w8i * w8i, w8i * w8i * w8i};
    Fr nf = Fr::zero();
    nf.v[0] = (uint32_t)(8 * n);
    nf.v[1] = (uint32_t)((8 * n) >> 32);
    const Fr inv8n = pnp::inverse(to_mont(nf));
    const Fr gni = pnp::inverse(pow_u64(host_gen(), n));
    Fr gn[8];
    gn[0] = Fr::one();
    for (int k = 1; k < 8; k++) gn[k] = gn[k - 1] * gni;
    TcombExt<M> ext;
    if (M < 8) {
        // rows m1 = M .. 7 of sum_m w_8^(-m m1) Y_m = 0: A [Y_M..Y_7] = -B [Y_0..Y_(M-1)],
        // Gauss-Jordan on [A | -B] (A is a Vandermonde block: invertible)
        constexpr int E = 8 - M;
        Fr G[E][8];
        for (int e = 0; e < E; e++) {
            const int m1 = M + e;
            for (int m = 0; m < 8; m++) {
                const Fr v = pow_u64(w8i, (uint64_t)((m * m1) % 8));
                if (m >= M) G[e][m - M] = v;
                else G[e][E + m] = Fr::zero() - v;
            }
        }
        for (int c = 0; c < E; c++) {
            int p = c;
            while (G[p][c].is_zero()) p++;
            if (p != c)
                for (int j = 0; j < 8; j++) std::swap(G[p][j], G[c][j]);
            const Fr inv = pnp::inverse(G[c][c]);
            for (int j = 0; j < 8; j++) G[c][j] = G[c][j] * inv;
            for (int r = 0; r < E; r++) {
                if (r == c || G[r][c].is_zero()) continue;
                const Fr f = G[r][c];
                for (int j = 0; j < 8; j++) G[r][j] = G[r][j] - f * G[c][j];
            }
        }
        for (int e = 0; e < E; e++)
            for (int m = 0; m < M; m++) ext.c[e * M + m] = G[e][E + m];
    }
    hipLaunchKernelGGL(k_t_combine<M>, dim3((uint32_t)((len + 255) / 256)), dim3(256), 0, s, Y, len, q0, out,
                       ext, w[1], w[2], w[3], inv8n, t.coset_inv_hi.u64(), t.coset_inv_lo.u64(), gn[0],
                       gn[1], gn[2], gn[3], gn[4], gn[5], gn[6], gn[7], nz);
    PNP_HIP(hipGetLastError());
}

void t_combine(NttTables &t, const uint64_t *Y, uint64_t len, uint64_t q0, uint64_t *out,
               uint32_t lg_n, unsigned *nz, hipStream_t s) {
    t_combine_m<8>(t, Y, len, q0, out, lg_n, nz, s);
}

void t_combine_blocks(NttTables &t, const uint64_t *Y, int nb, uint64_t *out, uint32_t lg_n, unsigned *nz,
                      hipStream_t s) {
    const uint64_t n = 1ULL << lg_n;
    switch (nb) {
        case 6: t_combine_m<6>(t, Y, n, 0, out, lg_n, nz, s); break;
        case 7: t_combine_m<7>(t, Y, n, 0, out, lg_n, nz, s); break;
        case 8: t_combine_m<8>(t, Y, n, 0, out, lg_n, nz, s); break;
        default:
            set_error("t_combine_blocks: %d blocks", nb);
            throw Error(PNP_E_ARG);
    }
}

// out[b n + brev(j)] = in[8 j + m0 + b], b < nb
// (natural 8n order -> block-bitrev layout, see lde_blocks)
__global__ void k_to_blocks(const uint64_t *in, uint64_t *out, uint64_t n, uint32_t lg_n, int m0, int nb) {
    uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint64_t p = lg_n ? brev((uint32_t)j, lg_n) : 0;
    for (int b = 0; b < nb; b++) store_fr(out, (uint64_t)b * n + p, load_fr(in, 8 * j + m0 + b));
}
void to_blocks(const uint64_t *in, uint64_t *out, uint32_t lg_n, int m0, int nb, hipStream_t s) {
    const uint64_t n = 1ULL << lg_n;
    hipLaunchKernelGGL(k_to_blocks, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, in, out, n, lg_n,
                       m0, nb);
    PNP_HIP(hipGetLastError());
}

}  // namespace pnp
