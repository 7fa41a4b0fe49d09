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

// ---------------------------------------------------------------------------
// The reference's own circuit: the HEIGHT-h Poseidon Merkle tree of
// merkle-tree/src/constraints.rs:20-107 (width-3 Poseidon, zprize_constraints.rs
// gadget, composer.rs zero-variable + blinding rows), laid out row for row like
// the reference composer (mirrors tests/merkle_circuit.py, which checks it):
//   row 0            zero_var constrained to 0 (q_l = 1)
//   rows 1..3        blinding (r1 r2 r3 r4), (r1' r2' r3' r4'), (r1' r2' 0 0)
//   hash p (193 rows from 4 + 193 p; bottom tree level first, root last):
//     r = 0..2       addi: (s_r, 0, A_r, 0), q_l = 1, q_c = rk[r], q_o = -1
//     r = 3+3k+j     round k (0..62), output j: (s0, s1, S_kj, s2), q_o = -1,
//                    full (k < 4 or k >= 59): q_hl q_hr q_h4 = M[j], q_c = rk[3k+3+j]
//                    (0 in the last round); partial: q_hl q_r q_4 = M[j], q_c idem
//     r = 192        assert_equal(node, S_62,1): (node, S, 0, 0), q_l = 1, q_r = -1
//   root row         (root, 0, 0, 0), q_l = 1, q_o = -1, PI = -root
// Copy cycles follow the reference's insertion order (row-major, wires
// l r o 4, permutation/mod.rs:114-131).  `pc` holds (Montgomery) rk[189], M[9]
// row-major, the domain tag.
namespace merkle {
constexpr int ROWS = 193, ROUNDS = 63, NRK = 189;
constexpr uint64_t FIRST = 4;  // rows before the first hash

// hash position of tree node i (level l = floor(log2(i + 1))): deeper levels first
__device__ __forceinline__ uint64_t hash_pos(uint64_t node, int H) {
    const int l = 63 - __builtin_clzll(node + 1);
    return (1ULL << (H - 1)) - (2ULL << l) + node - (1ULL << l) + 1;
}
__device__ __forceinline__ uint64_t node_of(uint64_t p, int H) {
    uint64_t cum = 0;
    for (int l = H - 2; l >= 0; l--) {
        const uint64_t cnt = 1ULL << l;
        if (p < cum + cnt) return cnt - 1 + (p - cum);
        cum += cnt;
    }
    return 0;
}
}  // namespace merkle

// one tree level: thread t hashes node (2^l - 1 + t) and writes its 193 rows
__global__ __launch_bounds__(64) void k_merkle_level_(int H, int l, const uint64_t *pc, const uint64_t *leaves,
                                                      uint64_t *nodes, uint64_t *w0, uint64_t *w1,
                                                      uint64_t *w2, uint64_t *w3) {
    using namespace merkle;
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (t >= (1ULL << l)) return;
    const uint64_t node = (1ULL << l) - 1 + t, nl = (1ULL << (H - 1)) - 1;
    const uint64_t base = FIRST + ROWS * hash_pos(node, H);
    const Fr zero = Fr::zero();
    auto row = [&](uint64_t r, const Fr &a, const Fr &b, const Fr &c, const Fr &d) {
        store_fr(w0, base + r, a);
        store_fr(w1, base + r, b);
        store_fr(w2, base + r, c);
        store_fr(w3, base + r, d);
    };
    auto rk = [&](int k) { return load_fr(pc, k); };
    auto M = [&](int j, int i) { return load_fr(pc, NRK + 3 * j + i); };
    auto p5 = [](const Fr &x) { Fr x2 = x * x; return x2 * x2 * x; };
    Fr s[3];
    s[0] = load_fr(pc, NRK + 9);
    s[1] = l == H - 2 ? load_fr(leaves, 2 * node + 1 - nl) : load_fr(nodes, 2 * node + 1);
    s[2] = l == H - 2 ? load_fr(leaves, 2 * node + 2 - nl) : load_fr(nodes, 2 * node + 2);
    for (int r = 0; r < 3; r++) {
        const Fr a = s[r] + rk(r);
        row(r, s[r], zero, a, zero);
        s[r] = a;
    }
    for (int k = 0; k < ROUNDS; k++) {
        const bool full = k < 4 || k >= ROUNDS - 4;
        const Fr e0 = p5(s[0]);
        const Fr e1 = full ? p5(s[1]) : s[1], e2 = full ? p5(s[2]) : s[2];
        Fr o[3];
        for (int j = 0; j < 3; j++) {
            o[j] = M(j, 0) * e0 + M(j, 1) * e1 + M(j, 2) * e2;
            if (k < ROUNDS - 1) o[j] = o[j] + rk(3 * k + 3 + j);
            row(3 + 3 * k + j, s[0], s[1], o[j], s[2]);
        }
        s[0] = o[0], s[1] = o[1], s[2] = o[2];
    }
    row(ROWS - 1, s[1], s[1], zero, zero);
    store_fr(nodes, node, s[1]);
}

// selectors and sigmas of every row of the domain (one thread per row)
__global__ void k_merkle_layout_(int H, uint64_t n, const uint64_t *pc, uint64_t *ql, uint64_t *qr,
                                 uint64_t *qo, uint64_t *q4, uint64_t *qc, uint64_t *qhl, uint64_t *qhr,
                                 uint64_t *qh4, uint64_t *qarith, uint64_t *s0, uint64_t *s1, uint64_t *s2,
                                 uint64_t *s3, Fr omega, Fr k1, Fr k2, Fr k3) {
    using namespace merkle;
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t NH = (1ULL << (H - 1)) - 1, root_row = FIRST + ROWS * NH;
    const Fr one = Fr::one(), m1 = neg(one), zero = Fr::zero();
    Fr sel[9] = {zero, zero, zero, zero, zero, zero, zero, zero, zero};  // ql qr qo q4 qc qhl qhr qh4 qarith
    // next slot of each wire of this row (row, wire); identity by default
    uint64_t nr[4] = {i, i, i, i};
    int nw[4] = {0, 1, 2, 3};
    auto to = [&](int w, uint64_t r, int w2) { nr[w] = r, nw[w] = w2; };
    const int WL = 0, WR = 1, WO = 2, W4 = 3;
    const int win[3] = {WL, WR, W4};  // the wire carrying state element x in a round row
    if (i == 0) {
        sel[0] = one, sel[8] = one;
        to(WL, 0, WR), to(WR, 0, WO), to(WO, 0, W4), to(W4, 3, WO);
    } else if (i == 2) {
        to(WL, 3, WL), to(WR, 3, WR);
    } else if (i == 3) {
        to(WL, 2, WL), to(WR, 2, WR), to(WO, 3, W4), to(W4, FIRST, WR);
    } else if (i >= FIRST && i < root_row) {
        const uint64_t p = (i - FIRST) / ROWS, hb = FIRST + ROWS * p;
        const int r = (int)(i - hb);
        const uint64_t node = node_of(p, H);
        const bool leaf_parent = node >= (1ULL << (H - 2)) - 1;
        if (r < 3) {  // addi
            sel[0] = one, sel[2] = m1, sel[4] = load_fr(pc, r), sel[8] = one;
            if (r > 0 && !leaf_parent) {  // a child node: its own assert row first
                const uint64_t c = 2 * node + r;
                to(WL, FIRST + ROWS * hash_pos(c, H) + ROWS - 1, WL);
            }
            to(WR, i, W4);
            to(W4, r < 2 ? i + 1 : hb + ROWS - 1, r < 2 ? WR : WO);
            to(WO, hb + 3, win[r]);
        } else if (r < ROWS - 1) {
            const int k = (r - 3) / 3, j = (r - 3) % 3;
            const bool full = k < 4 || k >= ROUNDS - 4;
            sel[5] = load_fr(pc, NRK + 3 * j);
            if (full) {
                sel[6] = load_fr(pc, NRK + 3 * j + 1), sel[7] = load_fr(pc, NRK + 3 * j + 2);
            } else {
                sel[1] = load_fr(pc, NRK + 3 * j + 1), sel[3] = load_fr(pc, NRK + 3 * j + 2);
            }
            if (k < ROUNDS - 1) sel[4] = load_fr(pc, 3 * k + 3 + j);
            sel[2] = m1, sel[8] = one;
            for (int x = 0; x < 3; x++) {
                const uint64_t producer = k == 0 ? hb + x : hb + 3 + 3 * (k - 1) + x;
                if (j < 2) to(win[x], i + 1, win[x]);
                else to(win[x], producer, WO);
            }
            if (k < ROUNDS - 1) to(WO, hb + 3 + 3 * (k + 1), win[j]);
            else if (j == 1) to(WO, hb + ROWS - 1, WR);
        } else {  // assert_equal(node, hash output)
            sel[0] = one, sel[1] = m1, sel[8] = one;
            if (node == 0) {
                to(WL, root_row, WL);
            } else {
                const uint64_t par = (node - 1) / 2;
                to(WL, FIRST + ROWS * hash_pos(par, H) + ((node & 1) ? 1 : 2), WL);
            }
            to(WR, hb + 3 + 3 * (ROUNDS - 1) + 1, WO);
            to(WO, i, W4);
            to(W4, p + 1 < NH ? hb + ROWS : root_row, WR);
        }
    } else if (i == root_row) {
        sel[0] = one, sel[2] = m1, sel[8] = one;
        to(WL, root_row - 1, WL), to(WR, i, WO), to(WO, i, W4), to(W4, 0, WL);
    }
    uint64_t *S[9] = {ql, qr, qo, q4, qc, qhl, qhr, qh4, qarith};
    for (int q = 0; q < 9; q++) store_fr(S[q], i, sel[q]);
    const Fr K[4] = {one, k1, k2, k3};
    uint64_t *SG[4] = {s0, s1, s2, s3};
    for (int w = 0; w < 4; w++) store_fr(SG[w], i, K[nw[w]] * pow_u64(omega, nr[w]));
}

void k_synth_merkle(int height, const uint64_t *pc_mont_host, const uint64_t *leaves, const uint64_t *blind,
                    uint64_t *nodes, uint64_t *const w[4], uint64_t *const sel[9], uint64_t *const sigma[4],
                    uint64_t n, hipStream_t s) {
    using namespace merkle;
    const uint64_t ng = FIRST + ROWS * ((1ULL << (height - 1)) - 1) + 1;
    if (height < 2 || height > 20 || ng > n) {
        set_error("synth_merkle: height %d needs %llu rows, domain %llu", height, (unsigned long long)ng,
                  (unsigned long long)n);
        throw Error(PNP_E_ARG);
    }
    uint32_t lg = 0;
    while ((1ULL << lg) < n) lg++;
    DevBuf pc((NRK + 10) * 32);
    PNP_HIP(hipMemcpyAsync(pc.p, pc_mont_host, (NRK + 10) * 32, hipMemcpyHostToDevice, s));
    // rows 0..3: zero row, blinding rows (r1 r2 r3 r4), (r1' r2' r3' r4'), (r1' r2' 0 0)
    for (int j = 0; j < 4; j++) PNP_HIP(hipMemsetAsync(w[j], 0, 32 * FIRST, s));
    for (int r = 1; r <= 2; r++)
        for (int j = 0; j < 4; j++)
            PNP_HIP(hipMemcpyAsync(w[j] + 4 * r, blind + 4 * (4 * (r - 1) + j), 32, hipMemcpyDeviceToDevice, s));
    for (int j = 0; j < 2; j++)
        PNP_HIP(hipMemcpyAsync(w[j] + 4 * 3, blind + 4 * (4 + j), 32, hipMemcpyDeviceToDevice, s));
    for (int l = height - 2; l >= 0; l--) {
        hipLaunchKernelGGL(k_merkle_level_, dim3(nblk(1ULL << l, 64)), dim3(64), 0, s, height, l, pc.u64(),
                           leaves, nodes, w[0], w[1], w[2], w[3]);
        PNP_HIP(hipGetLastError());
    }
    // root row (root, 0, 0, 0)
    const uint64_t rr = ng - 1;
    for (int j = 1; j < 4; j++) PNP_HIP(hipMemsetAsync(w[j] + 4 * rr, 0, 32, s));
    PNP_HIP(hipMemcpyAsync(w[0] + 4 * rr, nodes, 32, hipMemcpyDeviceToDevice, s));
    const uint64_t root32[4] = {13381757501831005802ULL, 6564924994866501612ULL, 789602057691799140ULL,
                                6625830629041353339ULL};
    Fr omega = pow_u64(from_u64_limbs<FrP>(root32), 1ULL << (32 - lg));
    auto fr_small = [](uint32_t v) { Fr r = Fr::zero(); r.v[0] = v; return to_mont(r); };
    hipLaunchKernelGGL(k_merkle_layout_, dim3(nblk(n)), dim3(256), 0, s, height, n, pc.u64(), sel[0], sel[1],
                       sel[2], sel[3], sel[4], sel[5], sel[6], sel[7], sel[8], sigma[0], sigma[1], sigma[2],
                       sigma[3], omega, fr_small(7), fr_small(13), fr_small(17));
    PNP_HIP(hipGetLastError());
    PNP_HIP(hipStreamSynchronize(s));  // pc is freed on return
}

}  // namespace pnp
