// wires.hip — the round-1 wire commitments over copy-constraint groups.
//
// The reference commits each wire polynomial from its coefficients
// (gen_proof.cuh:25-50); lagrange.hip already commits it from its padded
// evaluations, sum_i w_i L_i over the Lagrange-basis key.  A satisfying
// witness repeats values by construction: every position of one cycle of the
// copy permutation sigma holds the same variable.  In the reference's
// Poseidon Merkle circuit each full round keeps the state (s0, s1, s2) in
// wires a, b, d of three consecutive rows (zprize_constraints.rs:141-262,
// hash.rs:20-117), so those wires hold each value ~3 times: a wire has only
// ~1/3 as many distinct variables as rows.  With
//     B_{j,C} = sum_{i : (j, i) in C} L_i
// for every cycle C of sigma restricted to wire j (a "group"),
//     commit(w_j) = sum_i w_i L_i = sum_C w(C) B_{j,C}
// — the same group element, hence the same proof bytes, from one scalar per
// group: the MSM of a Merkle wire shrinks ~3x.
//
// The groups depend only on the prover key (sigma) and the bases only on the
// commit key (the Lagrange points): both are built once, on the first proof
// after either changes (like the folded tables), on the GPU:
//   1. sigma decoded into a successor permutation of the 4n positions
//      p = j n + i: sigma_j(w^i) = k_j' w^i' (K = 1, 7, 13, 17,
//      permutation/constants.cu:3-15) is looked up among the identity values
//      k_j w^i (a radix sort of their low 64 bits, full 256-bit compare);
//   2. every position labelled with the smallest position of its cycle
//      (pointer jumping, log2(4n) rounds);
//   3. per wire, rows sorted by label: runs = groups, each with a
//      representative row; run sums of the L_i (exact XYZZ additions, chunked
//      so large groups — the zero variable's — stay parallel) -> affine bases;
//   4. one folded table (msm_build_table) over the bases of all four wires,
//      MSM b reading its wire's n-slot segment (MsmSegs); group k sits at
//      slot bitrev(k) (wb_slot), so the groups spread over the whole segment
//      and every rank of a sharded MSM gets its share of them.
// A wire whose groups are nearly all single rows (g > 0.9 n, the Merkle
// circuit's wire c) keeps the plain Lagrange points as its segment: its
// scalars are its evaluations.
//
// Per proof: one kernel gathers each group's scalar from its representative
// row and checks that every row of the group holds the same value.  A witness
// that breaks a copy constraint (an unsatisfiable circuit) fails the check and
// the caller commits from the evaluations as before, so the commitments are
// exactly sum_i w_i L_i for every input.
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include "context.h"
#include "ec.cuh"
#include "protocol.h"

namespace pnp {

namespace {

inline uint32_t nblk(uint64_t threads, uint32_t bs = 256) { return (uint32_t)((threads + bs - 1) / bs); }

__device__ __forceinline__ bool fr_eq(const uint64_t *a, const uint64_t *b) {
    return a[0] == b[0] && a[1] == b[1] && a[2] == b[2] && a[3] == b[3];
}

__global__ void k_wb_keys(const uint64_t *idv, uint64_t N, uint64_t *key, uint32_t *pos) {
    const uint64_t p = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (p >= N) return;
    key[p] = idv[4 * p];
    pos[p] = (uint32_t)p;
}

struct SigmaPtrs {
    const uint64_t *s[4];
};

// next[p] = the position whose identity value equals sigma(p); *bad when
// sigma(p) is no identity value (not a permutation of the 4n positions)
__global__ void k_wb_next(SigmaPtrs sg, uint64_t n, const uint64_t *skey, const uint32_t *spos,
                          const uint64_t *idv, uint32_t *next, uint32_t *bad) {
    const uint64_t p = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t N = 4 * n;
    if (p >= N) return;
    const uint64_t *v = sg.s[p / n] + 4 * (p % n);
    const uint64_t k = v[0];
    uint64_t lo = 0, hi = N;  // first index with skey >= k
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (skey[mid] < k) lo = mid + 1;
        else hi = mid;
    }
    uint32_t q = (uint32_t)p;
    bool found = false;
    for (uint64_t t = lo; t < N && skey[t] == k; t++) {
        if (fr_eq(idv + 4 * (uint64_t)spos[t], v)) {
            q = spos[t];
            found = true;
            break;
        }
    }
    if (!found) atomicOr(bad, 1u);
    next[p] = q;
}

__global__ void k_wb_iota(uint32_t *a, uint64_t N) {
    const uint64_t p = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (p < N) a[p] = (uint32_t)p;
}

// one pointer-jumping round: lab = min over the next 2^(k+1) orbit positions
__global__ void k_wb_jump(const uint32_t *lab, const uint32_t *nx, uint32_t *lab2, uint32_t *nx2, uint64_t N) {
    const uint64_t p = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (p >= N) return;
    const uint32_t q = nx[p];
    lab2[p] = min(lab[p], lab[q]);
    nx2[p] = nx[q];
}

__global__ void k_wb_heads(const uint32_t *slab, uint64_t n, uint32_t *head) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (t < n) head[t] = (t == 0 || slab[t] != slab[t - 1]) ? 1u : 0u;
}

// group k sits at slot bitrev(k) of its wire's n-slot segment (n = 2^lg, k <
// g <= n): any run of consecutive groups spreads evenly over the segment, so
// every rank's point range of a sharded MSM (n / W slots) holds its share of
// them — the groups come in label order, the Merkle wires' real variables
// first and the padding rows' singletons last; packed at the front (or spread
// in order) the non-zero scalars would all fall to the first ranks
__device__ __forceinline__ uint32_t wb_slot(uint64_t k, uint64_t g, uint64_t n) {
    (void)g;
    const int lg = 63 - __clzll(n);
    return lg ? (uint32_t)(__brevll(k) >> (64 - lg)) : 0u;
}

// gid: inclusive scan of the heads (group index + 1)
__global__ void k_wb_groups(const uint32_t *srow, const uint32_t *gid, const uint32_t *head, uint64_t n,
                            uint64_t g_cnt, uint32_t *grp, uint32_t *rep, uint32_t *gstart) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (t >= n) return;
    const uint32_t g = gid[t] - 1, row = srow[t], slot = wb_slot(g, g_cnt, n);
    grp[row] = slot;
    if (head[t]) {
        rep[slot] = row;
        gstart[g] = (uint32_t)t;
    }
}

// run sums, level 1: lane c adds the L of sorted positions [c C, (c+1) C)
// and leaves the sum of every piece (a group's part inside the chunk) at the
// piece's last position
__global__ __launch_bounds__(256) void k_wb_chunks(const uint64_t *L, const uint32_t *srow, const uint32_t *gid,
                                                   uint64_t n, uint32_t C, uint64_t *part) {
    const uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t lo = c * C;
    if (lo >= n) return;
    const uint64_t hi = lo + C < n ? lo + C : n;
    Xyzz acc = Xyzz::inf();
#pragma unroll 1
    for (uint64_t t = lo; t < hi; t++) {
        const uint64_t *pt = L + 12 * (uint64_t)srow[t];
        acc = madd(acc, load_fq(pt), load_fq(pt + 6));
        if (t + 1 == hi || gid[t + 1] != gid[t]) {
            store_xyzz(part + 24 * t, acc);
            acc = Xyzz::inf();
        }
    }
}

// level 2: group g = the pieces ending at the chunk boundaries inside its run
// and at its last position; *bad when a base is infinity (a degenerate key).
// A group of more than WB_HEAVY pieces (z's run over the 1M padding rows of
// the HEIGHT = 15 circuit: 32K pieces, 0.68 s in one lane) is queued in
// heavy[1..] instead and summed by a whole workgroup (k_wb_final_heavy)
constexpr uint64_t WB_HEAVY = 256;
__device__ __forceinline__ uint64_t wb_piece_end(uint64_t t0, uint64_t t1, uint32_t C, uint64_t k) {
    const uint64_t e = (t0 / C + 1 + k) * C;
    return (e < t1 ? e : t1) - 1;  // last position of piece k
}
__global__ __launch_bounds__(256) void k_wb_final(const uint64_t *part, const uint32_t *gstart, uint64_t g_cnt,
                                                  uint64_t n, uint32_t C, uint64_t *out, uint32_t *bad,
                                                  uint32_t *heavy) {
    const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (g >= g_cnt) return;
    const uint64_t t0 = gstart[g], t1 = g + 1 < g_cnt ? gstart[g + 1] : n;
    const uint64_t np = (t1 - 1) / C - t0 / C + 1;  // pieces of the run
    if (np > WB_HEAVY) {
        heavy[1 + atomicAdd(heavy, 1u)] = (uint32_t)g;
        return;
    }
    Xyzz acc = Xyzz::inf();
#pragma unroll 1
    for (uint64_t k = 0; k < np; k++) acc = add(acc, load_xyzz(part + 24 * wb_piece_end(t0, t1, C, k)));
    if (acc.is_inf()) atomicOr(bad, 1u);
    store_xyzz(out + 24 * (uint64_t)wb_slot(g, g_cnt, n), acc);
}
// the queued heavy groups, one workgroup each (strided partial sums, then a
// tree in LDS); the grid strides over the queue, whose length stays on the device
__global__ __launch_bounds__(256) void k_wb_final_heavy(const uint64_t *part, const uint32_t *gstart, uint64_t g_cnt,
                                                        uint64_t n, uint32_t C, uint64_t *out, uint32_t *bad,
                                                        const uint32_t *heavy) {
    __shared__ Xyzz red[256];
    for (uint32_t q = blockIdx.x; q < heavy[0]; q += gridDim.x) {
        const uint64_t g = heavy[1 + q];
        const uint64_t t0 = gstart[g], t1 = g + 1 < g_cnt ? gstart[g + 1] : n;
        const uint64_t np = (t1 - 1) / C - t0 / C + 1;
        Xyzz acc = Xyzz::inf();
#pragma unroll 1
        for (uint64_t k = threadIdx.x; k < np; k += blockDim.x)
            acc = add(acc, load_xyzz(part + 24 * wb_piece_end(t0, t1, C, k)));
        red[threadIdx.x] = acc;
        __syncthreads();
        for (uint32_t h = blockDim.x / 2; h > 0; h /= 2) {
            if (threadIdx.x < h) red[threadIdx.x] = add(red[threadIdx.x], red[threadIdx.x + h]);
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            if (red[0].is_inf()) atomicOr(bad, 1u);
            store_xyzz(out + 24 * (uint64_t)wb_slot(g, g_cnt, n), red[0]);
        }
        __syncthreads();
    }
}

// z's runs: z_(i+1) = z_i ratio_i and ratio_i = 1 exactly when sigma fixes
// all four positions of row i (the numerator and denominator products are the
// same expression), so a run of fixed rows continues z's run; a run starts at
// row 0 and after every row that sigma moves
__global__ void k_wb_zheads(const uint32_t *next, uint64_t n, uint32_t *head, uint32_t *row) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    bool cont = i > 0;
    for (int j = 0; j < 4 && cont; j++) {
        const uint64_t p = (uint64_t)j * n + i - 1;
        cont = next[p] == (uint32_t)p;
    }
    head[i] = cont ? 0u : 1u;
    row[i] = (uint32_t)i;
}

// Lagrange points (affine) -> XYZZ, for an ungrouped wire's segment
__global__ void k_wb_lift(const uint64_t *L, uint64_t n, uint64_t *out) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    Xyzz p;
    p.x = load_fq(L + 12 * i);
    p.y = load_fq(L + 12 * i + 6);
    p.zz = Fq::one();
    p.zzz = Fq::one();
    store_xyzz(out + 24 * i, p);
}

struct WirePtrs {
    const uint64_t *w[4];
    const uint32_t *grp[4], *rep[4];
    uint64_t *scal[4];
};

// per proof: scal_j[g] = w_j[rep_j[g]]; any row differing from its group's
// representative sets *flag
__global__ void k_wb_gather(WirePtrs wp, uint64_t n, uint32_t *flag) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const int j = blockIdx.y;
    if (i >= n || !wp.grp[j]) return;
    const uint32_t g = wp.grp[j][i], r = wp.rep[j][g];
    const uint64_t *v = wp.w[j] + 4 * i;
    if (r == i) {
#pragma unroll
        for (int k = 0; k < 4; k++) wp.scal[j][4 * (uint64_t)g + k] = v[k];
    } else if (!fr_eq(v, wp.w[j] + 4 * (uint64_t)r)) {
        atomicOr(flag, 1u);
    }
}

bool groups_enabled() {
    static const bool v = [] {
        const char *e = getenv("PNP_WIRE_GROUPS");
        return !e || atoi(e) != 0;
    }();
    return v;
}
bool z_groups_enabled() {
    static const bool v = [] {
        const char *e = getenv("PNP_Z_GROUPS");
        return !e || atoi(e) != 0;
    }();
    return v && groups_enabled();
}

// hipcub temporary storage, grown on demand
void *cub_tmp(DevBuf &b, size_t bytes) {
    if (b.bytes < bytes) b.alloc(bytes);
    return b.p;
}

// the groups and bases of the resident keys (n a power of two, lag_points of
// size n present); sets wb.ok
void build_wire_bases(pnp_ctx *ctx, uint64_t n) {
    auto &wb = ctx->wb;
    hipStream_t s = tables_stream(ctx);
    wb = pnp_ctx::WireBases{};
    wb.built = true;
    wb.n = n;
    wb.pk_gen = ctx->pk_gen;
    uint32_t lg = 0;
    while ((1ULL << lg) < n) lg++;
    const uint64_t N = 4 * n;
    DevBuf flag(16), tmp;
    uint32_t *bad = static_cast<uint32_t *>(flag.p);
    PNP_HIP(hipMemsetAsync(bad, 0, 4, s));
    // the sigma evaluations this build reads, kept to recognise the key later
    wb.sigma.alloc(N * 32);
    for (int j = 0; j < 4; j++)
        PNP_HIP(hipMemcpyAsync(wb.sigma.u64() + 4 * (uint64_t)j * n, ctx->pk_sigma_n[j].u64(), n * 32,
                               hipMemcpyDeviceToDevice, s));
    // 1. successor of every position
    DevBuf next(N * 4), lab(N * 4);
    {
        DevBuf idv(N * 32), key(N * 8), key2(N * 8), pos(N * 4), pos2(N * 4);
        const uint64_t kv[4] = {1, 7, 13, 17};
        for (int j = 0; j < 4; j++)
            k_geometric(idv.u64() + 4 * (uint64_t)j * n, n, fr_from_u64(kv[j]), root_of_unity(lg), s);
        hipLaunchKernelGGL(k_wb_keys, dim3(nblk(N)), dim3(256), 0, s, idv.u64(), N, key.u64(),
                           static_cast<uint32_t *>(pos.p));
        PNP_HIP(hipGetLastError());
        bg_step(s);
        size_t tb = 0;
        PNP_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, key.u64(), key2.u64(),
                                                   static_cast<uint32_t *>(pos.p), static_cast<uint32_t *>(pos2.p),
                                                   (int)N, 0, 64, s));
        PNP_HIP(hipcub::DeviceRadixSort::SortPairs(cub_tmp(tmp, tb), tb, key.u64(), key2.u64(),
                                                   static_cast<uint32_t *>(pos.p), static_cast<uint32_t *>(pos2.p),
                                                   (int)N, 0, 64, s));
        SigmaPtrs sg;
        for (int j = 0; j < 4; j++) sg.s[j] = wb.sigma.u64() + 4 * (uint64_t)j * n;
        hipLaunchKernelGGL(k_wb_next, dim3(nblk(N)), dim3(256), 0, s, sg, n, key2.u64(),
                           static_cast<const uint32_t *>(pos2.p), idv.u64(), static_cast<uint32_t *>(next.p), bad);
        PNP_HIP(hipGetLastError());
        bg_step(s);
    }
    // 2. cycle labels (the jumps run on a copy: `next` stays the successor,
    // z's runs below read it)
    {
        DevBuf lab2(N * 4), nx1(N * 4), nx2(N * 4);
        PNP_HIP(hipMemcpyAsync(nx1.p, next.p, N * 4, hipMemcpyDeviceToDevice, s));
        uint32_t *la = static_cast<uint32_t *>(lab.p), *lb = static_cast<uint32_t *>(lab2.p);
        uint32_t *na = static_cast<uint32_t *>(nx1.p), *nb = static_cast<uint32_t *>(nx2.p);
        hipLaunchKernelGGL(k_wb_iota, dim3(nblk(N)), dim3(256), 0, s, la, N);
        PNP_HIP(hipGetLastError());
        bg_step(s);
        for (uint64_t span = 1; span < N; span *= 2) {
            hipLaunchKernelGGL(k_wb_jump, dim3(nblk(N)), dim3(256), 0, s, la, na, lb, nb, N);
            PNP_HIP(hipGetLastError());
            bg_step(s);
            std::swap(la, lb);
            std::swap(na, nb);
        }
        if (la != static_cast<uint32_t *>(lab.p))
            PNP_HIP(hipMemcpyAsync(lab.p, la, N * 4, hipMemcpyDeviceToDevice, s));
    }
    // 3. per wire: groups, representatives, run sums of the Lagrange points
    const uint64_t *L = ctx->lag_points.u64();
    std::vector<DevBuf> bx(5);
    {
        DevBuf srt(n * 4), srow(n * 4), row(n * 4), head(n * 4), gid(n * 4), gstart(n * 4), part(n * 192);
        // a group of more than WB_HEAVY pieces spans at least (WB_HEAVY - 1) C + 2
        // positions (its first and last pieces may hold one each), so at most
        // n / ((WB_HEAVY - 1) C) of them are queued, + the count word
        DevBuf heavy((n / (32 * (WB_HEAVY - 1)) + 2) * 4);
        uint32_t *srt_p = static_cast<uint32_t *>(srt.p), *srow_p = static_cast<uint32_t *>(srow.p);
        uint32_t *head_p = static_cast<uint32_t *>(head.p), *gid_p = static_cast<uint32_t *>(gid.p);
        const int bits = (int)lg + 2;  // labels < 4n
        const uint32_t C = 32;
        // groups (rows srow in group order, heads, gid = inclusive scan) ->
        // slots, representatives and the run sums of the Lagrange points
        auto bases = [&](int j, uint32_t g) {
            wb.grp[j].alloc(n * 4);
            wb.rep[j].alloc(n * 4);
            hipLaunchKernelGGL(k_wb_groups, dim3(nblk(n)), dim3(256), 0, s, srow_p, gid_p, head_p, n, (uint64_t)g,
                               static_cast<uint32_t *>(wb.grp[j].p), static_cast<uint32_t *>(wb.rep[j].p),
                               static_cast<uint32_t *>(gstart.p));
            PNP_HIP(hipGetLastError());
            bg_step(s);
            hipLaunchKernelGGL(k_wb_chunks, dim3(nblk((n + C - 1) / C)), dim3(256), 0, s, L, srow_p, gid_p, n, C,
                               part.u64());
            PNP_HIP(hipGetLastError());
            bg_step(s);
            // the n slots: valid points everywhere (the empty slots' are never
            // read, their scalars stay zero), the group sums at the group slots
            bx[j].alloc(n * 192);
            hipLaunchKernelGGL(k_wb_lift, dim3(nblk(n)), dim3(256), 0, s, L, n, bx[j].u64());
            PNP_HIP(hipGetLastError());
            bg_step(s);
            PNP_HIP(hipMemsetAsync(heavy.p, 0, 4, s));
            hipLaunchKernelGGL(k_wb_final, dim3(nblk(g)), dim3(256), 0, s, part.u64(),
                               static_cast<const uint32_t *>(gstart.p), (uint64_t)g, n, C, bx[j].u64(), bad,
                               static_cast<uint32_t *>(heavy.p));
            PNP_HIP(hipGetLastError());
            hipLaunchKernelGGL(k_wb_final_heavy, dim3(64), dim3(256), 0, s, part.u64(),
                               static_cast<const uint32_t *>(gstart.p), (uint64_t)g, n, C, bx[j].u64(), bad,
                               static_cast<const uint32_t *>(heavy.p));
            PNP_HIP(hipGetLastError());
            bg_step(s);
        };
        for (int j = 0; j < 4; j++) {
            const uint32_t *labj = static_cast<const uint32_t *>(lab.p) + (uint64_t)j * n;
            hipLaunchKernelGGL(k_wb_iota, dim3(nblk(n)), dim3(256), 0, s, static_cast<uint32_t *>(row.p), n);
            PNP_HIP(hipGetLastError());
            bg_step(s);
            size_t tb = 0;
            PNP_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, labj, srt_p, static_cast<uint32_t *>(row.p),
                                                       srow_p, (int)n, 0, bits, s));
            PNP_HIP(hipcub::DeviceRadixSort::SortPairs(cub_tmp(tmp, tb), tb, labj, srt_p,
                                                       static_cast<uint32_t *>(row.p), srow_p, (int)n, 0, bits, s));
            hipLaunchKernelGGL(k_wb_heads, dim3(nblk(n)), dim3(256), 0, s, srt_p, n, head_p);
            PNP_HIP(hipGetLastError());
            bg_step(s);
            tb = 0;
            PNP_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, tb, head_p, gid_p, (int)n, s));
            PNP_HIP(hipcub::DeviceScan::InclusiveSum(cub_tmp(tmp, tb), tb, head_p, gid_p, (int)n, s));
            uint32_t g = 0;
            PNP_HIP(hipMemcpyAsync(&g, gid_p + n - 1, 4, hipMemcpyDeviceToHost, s));
            PNP_HIP(hipStreamSynchronize(s));
            wb.g[j] = g;
            wb.ident[j] = (uint64_t)g * 10 > 9 * n;
            if (wb.ident[j]) {
                wb.g[j] = n;
                bx[j].alloc(n * 192);
                hipLaunchKernelGGL(k_wb_lift, dim3(nblk(n)), dim3(256), 0, s, L, n, bx[j].u64());
                PNP_HIP(hipGetLastError());
                bg_step(s);
                continue;
            }
            bases(j, g);
        }
        // z (segment 4): runs of rows sigma fixes, already in row order
        {
            hipLaunchKernelGGL(k_wb_zheads, dim3(nblk(n)), dim3(256), 0, s, static_cast<const uint32_t *>(next.p), n,
                               head_p, srow_p);
            PNP_HIP(hipGetLastError());
            bg_step(s);
            size_t tb = 0;
            PNP_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, tb, head_p, gid_p, (int)n, s));
            PNP_HIP(hipcub::DeviceScan::InclusiveSum(cub_tmp(tmp, tb), tb, head_p, gid_p, (int)n, s));
            uint32_t g = 0;
            PNP_HIP(hipMemcpyAsync(&g, gid_p + n - 1, 4, hipMemcpyDeviceToHost, s));
            PNP_HIP(hipStreamSynchronize(s));
            wb.g[4] = g;
            wb.ident[4] = (uint64_t)g * 10 > 9 * n;  // (not worth a segment: z commits from its evaluations)
            if (!wb.ident[4]) bases(4, g);
        }
    }
    uint32_t hbad = 0;
    PNP_HIP(hipMemcpyAsync(&hbad, bad, 4, hipMemcpyDeviceToHost, s));
    PNP_HIP(hipStreamSynchronize(s));
    // the wires are worth their segments only when some wire has far fewer
    // groups than rows; z when its runs merge >= 10% of the rows
    bool gain = false;
    for (int j = 0; j < 4; j++) gain |= !wb.ident[j] && wb.g[j] * 4 < 3 * n;
    wb.wires_ok = gain && !hbad;
    wb.z_ok = !wb.ident[4] && !hbad;
    if (!wb.wires_ok)
        for (int j = 0; j < 4; j++) {
            wb.grp[j].release();
            wb.rep[j].release();
            bx[j].release();
        }
    if (!wb.z_ok) {
        wb.grp[4].release();
        wb.rep[4].release();
        bx[4].release();
    }
    if (!wb.wires_ok && !wb.z_ok) return;  // wb.ok stays false (kept with its sigma): commit from the evaluations
    // 4. affine bases of the n-slot segments (wires a..d, z), one folded table;
    // multi-GPU point ranges (no bucket ranges): only this rank's slice
    // [p0, p1) of every segment, which is all its MSM share reads
    wb.sliced = ctx->msm.world > 1 && !ctx->msm.full_table();
    uint64_t p0 = 0, p1 = n;
    if (wb.sliced) msm_point_range(n, ctx->msm.rank, ctx->msm.world, p0, p1);
    const uint64_t sl = p1 - p0;
    wb.total = 0;
    for (int j = 0; j < 5; j++) {
        if (j < 4 ? !wb.wires_ok : !wb.z_ok) continue;
        wb.off[j] = wb.total;
        wb.total += sl;
    }
    wb.m = n;
    // the windows of ONE segment's MSM (n points), not of the whole table
    wb.c = msm_fold_c(n, ctx->msm.fold_c);
    if (wb.total) {
        DevBuf xyzz(wb.total * 192), aff(wb.total * 96);
        for (int j = 0; j < 5; j++) {
            if (!bx[j].p) continue;
            PNP_HIP(hipMemcpyAsync(xyzz.u64() + 24 * wb.off[j], bx[j].u64() + 24 * p0, sl * 192,
                                   hipMemcpyDeviceToDevice, s));
        }
        PNP_HIP(hipStreamSynchronize(s));
        for (auto &b : bx) b.release();
        xyzz_to_affine_dev(xyzz.u64(), wb.total, aff.u64(), s);
        xyzz.release();
        msm_build_table(wb.table, aff.u64(), wb.total, wb.c, s);
    }
    // every MSM of the batch reads n scalars: an ungrouped wire's evaluations,
    // a grouped wire's group values at their slots (zero elsewhere)
    wb.len = n;
    for (int j = 0; j < 5; j++) {
        if (wb.ident[j] || !wb.grp[j].p) continue;
        wb.scal[j].alloc(wb.len * 32);
        PNP_HIP(hipMemsetAsync(wb.scal[j].p, 0, wb.len * 32, s));
    }
    wb.flag.alloc(16);
    PNP_HIP(hipStreamSynchronize(s));
    wb.ok = true;
}

// the groups for domain n, (re)built when the keys changed
bool wire_bases_ready(pnp_ctx *ctx, uint64_t n) {
    if (tables_busy(ctx)) return false;  // being built in the background: commit without them
    auto &wb = ctx->wb;
    if (wb.built && wb.n == n && wb.pk_gen != ctx->pk_gen) {
        // the prover key was loaded again (the v1 symbol does it every call):
        // same sigma, same groups
        DevBuf own;  // (the builder's thread keeps off the proof's scratch)
        DevBuf &scr = t_bg_build ? own : ctx->scratch_b;
        bool same = wb.sigma.p != nullptr;
        for (int j = 0; j < 4 && same; j++)
            same = !k_any_diff(wb.sigma.u64() + 4 * (uint64_t)j * n, ctx->pk_sigma_n[j].u64(), 4 * n, scr,
                               tables_stream(ctx));
        if (same) wb.pk_gen = ctx->pk_gen;
        else wb.built = false;
    }
    // a deferring proof goes without them (built in the background or by the next proof)
    if ((!wb.built || wb.n != n) && ctx->defer_now && !t_bg_build) {
        ctx->tables_wanted = true;
        return false;
    }
    if (!wb.built || wb.n != n) {
        // built on the same call on every rank; a rank whose HBM cannot hold
        // the groups makes every rank commit without them
        bool fits = true;
        try {
            build_wire_bases(ctx, n);
        } catch (const Error &e) {
            if (e.code != PNP_E_NOMEM) throw;
            fits = false;
        }
        const bool all = all_ranks_ok(ctx, fits);
        if (!all) {
            ctx->wb = pnp_ctx::WireBases{};
            wb.built = true;
            wb.n = n;
            wb.pk_gen = ctx->pk_gen;
            ctx->hbm_groups_off = true;
        } else if (ctx->msm.world > 1) {  // the ranks' verdicts come from the same key: check they agree
            const bool w = all_ranks_ok(ctx, wb.wires_ok), z = all_ranks_ok(ctx, wb.z_ok);
            if (w != wb.wires_ok || z != wb.z_ok) {
                set_error("wire groups: the ranks built different groups from one prover key");
                throw Error(PNP_E_DEVICE);
            }
        }
    }
    return wb.ok;
}

}  // namespace

void wire_bases_reset(pnp_ctx *ctx) { ctx->wb = pnp_ctx::WireBases{}; }
void wire_bases_build(pnp_ctx *ctx, uint64_t n) {
    if (groups_enabled() && !ctx->hbm_groups_off) wire_bases_ready(ctx, n);
}
bool wire_groups_enabled() { return groups_enabled(); }

bool commit_wires_grouped(pnp_ctx *ctx, const uint64_t *const *d_evals, uint64_t n, CommitmentC *const *out) {
    if (!groups_enabled() || ctx->hbm_groups_off || !lagrange_table(ctx, n) || !wire_bases_ready(ctx, n) ||
        !ctx->wb.wires_ok)
        return false;
    auto &wb = ctx->wb;
    hipStream_t s = ctx->stream;
    uint32_t *flag = static_cast<uint32_t *>(wb.flag.p);
    PNP_HIP(hipMemsetAsync(flag, 0, 4, s));
    WirePtrs wp{};
    for (int j = 0; j < 4; j++) {
        wp.w[j] = d_evals[j];
        if (wb.ident[j]) continue;
        wp.grp[j] = static_cast<const uint32_t *>(wb.grp[j].p);
        wp.rep[j] = static_cast<const uint32_t *>(wb.rep[j].p);
        wp.scal[j] = wb.scal[j].u64();
    }
    hipLaunchKernelGGL(k_wb_gather, dim3(nblk(n), 4), dim3(256), 0, s, wp, n, flag);
    PNP_HIP(hipGetLastError());
    uint32_t hflag = 0;
    PNP_HIP(hipMemcpyAsync(&hflag, flag, 4, hipMemcpyDeviceToHost, s));
    PNP_HIP(hipStreamSynchronize(s));
    if (hflag) {  // a copy constraint does not hold: commit every row
        if (ctx->ktimer.enabled) ctx->ktimer.credit("wire_group_fallback", 1);
        return false;
    }
    const uint64_t *sc[4];
    MsmSegs segs;
    segs.n_table = wb.total;
    segs.sliced = wb.sliced;
    segs.c = wb.c;
    for (int j = 0; j < 4; j++) {
        sc[j] = wb.ident[j] ? d_evals[j] : wb.scal[j].u64();
        segs.off[j] = wb.off[j];
    }
    std::vector<uint64_t> xyzz(4 * 24);
    msm_run_batch(ctx->msm, nullptr, sc, 4, wb.len, xyzz.data(), s, wb.table.u64(), false, &segs);
    std::vector<uint64_t> aff(4 * 12);
    xyzz_to_affine_batch_host(xyzz.data(), 4, aff.data());
    for (int b = 0; b < 4; b++) {
        memcpy(out[b]->x, &aff[12 * b], 48);
        memcpy(out[b]->y, &aff[12 * b + 6], 48);
    }
    if (ctx->ktimer.enabled) ctx->ktimer.credit("wire_groups_used", 1);
    return true;
}

bool commit_z_grouped(pnp_ctx *ctx, const uint64_t *d_z, uint64_t n, CommitmentC *out) {
    if (!z_groups_enabled() || ctx->hbm_groups_off || !lagrange_table(ctx, n) || !wire_bases_ready(ctx, n) ||
        !ctx->wb.z_ok)
        return false;
    auto &wb = ctx->wb;
    hipStream_t s = ctx->stream;
    uint32_t *flag = static_cast<uint32_t *>(wb.flag.p);
    PNP_HIP(hipMemsetAsync(flag, 0, 4, s));
    WirePtrs wp{};
    wp.w[0] = d_z;
    wp.grp[0] = static_cast<const uint32_t *>(wb.grp[4].p);
    wp.rep[0] = static_cast<const uint32_t *>(wb.rep[4].p);
    wp.scal[0] = wb.scal[4].u64();
    hipLaunchKernelGGL(k_wb_gather, dim3(nblk(n), 1), dim3(256), 0, s, wp, n, flag);
    PNP_HIP(hipGetLastError());
    uint32_t hflag = 0;
    PNP_HIP(hipMemcpyAsync(&hflag, flag, 4, hipMemcpyDeviceToHost, s));
    PNP_HIP(hipStreamSynchronize(s));
    if (hflag) {  // (a zero denominator: the ratio of a fixed row was not 1)
        if (ctx->ktimer.enabled) ctx->ktimer.credit("z_group_fallback", 1);
        return false;
    }
    const uint64_t *sc[1] = {wb.scal[4].u64()};
    MsmSegs segs;
    segs.n_table = wb.total;
    segs.sliced = wb.sliced;
    segs.c = wb.c;
    segs.off[0] = wb.off[4];
    uint64_t xyzz[24], aff[12];
    msm_run_batch(ctx->msm, nullptr, sc, 1, wb.len, xyzz, s, wb.table.u64(), false, &segs);
    xyzz_to_affine_batch_host(xyzz, 1, aff);
    memcpy(out->x, aff, 48);
    memcpy(out->y, aff + 6, 48);
    if (ctx->ktimer.enabled) ctx->ktimer.credit("z_groups_used", 1);
    return true;
}

}  // namespace pnp
