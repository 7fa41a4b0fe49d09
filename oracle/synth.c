/*
 * oracle/synth.c — CPU mirror of the synthetic-instance generators of the
 * HIP library (zprize23-gpu-submission_amd/csrc/synth.hip, poly.hip
 * k_random_fr_), so a full-size (n = 2^22) instance that bench.py builds on
 * the GPU can be rebuilt here and proved by the CPU restatement.
 * TEST INFRASTRUCTURE ONLY (see pnp_oracle.h).
 *
 * These are not reference functions: they generate inputs (a satisfying
 * random arithmetic circuit of the Merkle circuit's shape, SURVEY 8(d)
 * config 4), and tests/test_gpu_prove.py checks GPU == CPU generation.
 */
#include "oracle_internal.h"

static inline uint64_t splitmix(uint64_t x) {
    x += 0x9e3779b97f4a7c15ULL;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
    return x ^ (x >> 31);
}

/* k_random_fr_: 4 splitmix words, top bit cleared, reduced once; the value is
 * used directly as a Montgomery residue */
void or_synth_random_fr(uint64_t *d, uint64_t n, uint64_t seed) {
#pragma omp parallel for schedule(static)
    for (int64_t ii = 0; ii < (int64_t)n; ii++) {
        uint64_t i = (uint64_t)ii, h = seed * 0x2545F4914F6CDD1DULL + i * 4, r[4];
        for (int k = 0; k < 4; k++) r[k] = splitmix(h + k);
        r[3] &= 0x7fffffffffffffffULL;
        if (!or_gt_n(OR_FR_P, r, 4)) {  /* r >= p: subtract once */
            unsigned __int128 br = 0;
            for (int k = 0; k < 4; k++) {
                unsigned __int128 t = (unsigned __int128)r[k] - OR_FR_P[k] - (uint64_t)br;
                r[k] = (uint64_t)t;
                br = (t >> 64) & 1;
            }
        }
        memcpy(d + 4 * i, r, 32);
    }
}

static uint64_t gcd64(uint64_t x, uint64_t y) {
    while (y) { uint64_t t = x % y; x = y; y = t; }
    return x;
}

/* k_synth_circuit (synth.hip): w[0] = a (in), w[1] = b, w[2] = c (out),
 * w[3] = d (in); sel[0..7] = q_l q_r q_o q_4 q_c q_hl q_hr q_h4 (in, n rows),
 * sel[8] = q_arith (out); sigma[0..3] out (n rows, Montgomery) */
void or_synth_circuit(uint64_t *const w[4], uint64_t *const sel[9], uint64_t *const sigma[4],
                      uint64_t n, uint64_t ng, uint64_t pi_pos, const uint64_t pi_canon[4]) {
    uint64_t A = 0x9E3779B1ULL % ng;
    if (ng <= 2) A = 1;
    while (gcd64(A, ng) != 1) A++;
    uint32_t lg = 0;
    while ((1ULL << lg) < n) lg++;
    uint64_t omega[4], k1[4], k2[4], k3[4], pi[4];
    or_root_of_unity(omega, lg);
    or_fr_from_u64(k1, 7);
    or_fr_from_u64(k2, 13);
    or_fr_from_u64(k3, 17);
    or_fr_to_mont(pi, pi_canon);
    /* sigma_0 is written at row pi(i) by row i: fill the identity part first */
    const int64_t CH = 1024;
#pragma omp parallel for schedule(static)
    for (int64_t c = 0; c < (int64_t)((n + CH - 1) / CH); c++) {
        uint64_t lo = (uint64_t)c * CH, hi = lo + CH < n ? lo + CH : n, wi[4];
        or_fr_pow(wi, omega, lo);
        for (uint64_t i = lo; i < hi; i++) {
            or_fr_mul(sigma[2] + 4 * i, k2, wi);
            or_fr_mul(sigma[3] + 4 * i, k3, wi);
            if (i >= ng) {
                fr_copy(sigma[0] + 4 * i, wi);
                or_fr_mul(sigma[1] + 4 * i, k1, wi);
                fr_zero(sel[8] + 4 * i);
            }
            or_fr_mul(wi, wi, omega);
        }
    }
#pragma omp parallel for schedule(static)
    for (int64_t c = 0; c < (int64_t)((ng + CH - 1) / CH); c++) {
        uint64_t lo = (uint64_t)c * CH, hi = lo + CH < ng ? lo + CH : ng, wi[4];
        or_fr_pow(wi, omega, lo);
        for (uint64_t i = lo; i < hi; i++) {
            uint64_t pii = (uint64_t)(((unsigned __int128)A * i + 1) % ng);
            const uint64_t *ai = w[0] + 4 * i, *bi = w[0] + 4 * pii, *di = w[3] + 4 * i;
            fr_copy(w[1] + 4 * i, bi);
            or_fr_pow(sigma[1] + 4 * i, omega, pii);
            or_fr_mul(sigma[0] + 4 * pii, k1, wi);
            uint64_t acc[4], t[4], p[4], x2[4];
            or_fr_mul(acc, sel[0] + 4 * i, ai);
            or_fr_mul(t, sel[1] + 4 * i, bi); or_fr_add(acc, acc, t);
            or_fr_mul(t, sel[3] + 4 * i, di); or_fr_add(acc, acc, t);
            const uint64_t *vv[3] = {ai, bi, di};
            for (int j = 0; j < 3; j++) {
                or_fr_mul(x2, vv[j], vv[j]);
                or_fr_mul(p, x2, x2);
                or_fr_mul(p, p, vv[j]);
                or_fr_mul(t, sel[5 + j] + 4 * i, p);
                or_fr_add(acc, acc, t);
            }
            or_fr_add(acc, acc, sel[4] + 4 * i);
            if (i == pi_pos) or_fr_add(acc, acc, pi);
            or_fr_neg(acc, acc);
            or_fr_inv(t, sel[2] + 4 * i);
            or_fr_mul(w[2] + 4 * i, acc, t);
            fr_copy(sel[8] + 4 * i, OR_FR_ONE);
            or_fr_mul(wi, wi, omega);
        }
    }
}

/* ------------------------------------------------------------------------
 * The reference's Poseidon Merkle circuit (k_synth_merkle, synth.hip; the row
 * layout of tests/merkle_circuit.py, which restates merkle-tree/src/
 * constraints.rs:20-107 + plonk-hashing zprize_constraints.rs:141-262 +
 * composer.rs:210-249,604-685).  pc = 199 Montgomery constants: rk[189],
 * MDS[9] row-major, domain tag.  Rows: 0 zero_var, 1..3 blinding, then 193
 * rows per hash (deepest level first), then the root row. */
#define MK_ROWS 193
#define MK_ROUNDS 63
#define MK_NRK 189
#define MK_FIRST 4

static uint64_t mk_hash_pos(uint64_t node, int H) {
    int l = 63 - __builtin_clzll(node + 1);
    return (1ULL << (H - 1)) - (2ULL << l) + node - (1ULL << l) + 1;
}

static uint64_t mk_node_of(uint64_t p, int H) {
    uint64_t cum = 0;
    for (int l = H - 2; l >= 0; l--) {
        uint64_t cnt = 1ULL << l;
        if (p < cum + cnt) return cnt - 1 + (p - cum);
        cum += cnt;
    }
    return 0;
}

static void mk_pow5(uint64_t r[4], const uint64_t x[4]) {
    uint64_t x2[4], x4[4];
    or_fr_mul(x2, x, x);
    or_fr_mul(x4, x2, x2);
    or_fr_mul(r, x4, x);
}

/* one hash gadget: node's 193 rows of the four wires, the output in nodes[node] */
static void mk_hash_rows(int H, uint64_t node, const uint64_t *pc, const uint64_t *leaves, uint64_t *nodes,
                         uint64_t *const w[4]) {
    const uint64_t nl = (1ULL << (H - 1)) - 1, base = MK_FIRST + MK_ROWS * mk_hash_pos(node, H);
    const int l = 63 - __builtin_clzll(node + 1);
    const uint64_t zero[4] = {0, 0, 0, 0};
#define MK_ROW(r, A, B, Cc, D) do { fr_copy(w[0] + 4 * (base + (r)), A); fr_copy(w[1] + 4 * (base + (r)), B); \
        fr_copy(w[2] + 4 * (base + (r)), Cc); fr_copy(w[3] + 4 * (base + (r)), D); } while (0)
    uint64_t s[3][4], o[3][4], e[3][4], t[4];
    fr_copy(s[0], pc + 4 * (MK_NRK + 9));
    if (l == H - 2) {
        fr_copy(s[1], leaves + 4 * (2 * node + 1 - nl));
        fr_copy(s[2], leaves + 4 * (2 * node + 2 - nl));
    } else {
        fr_copy(s[1], nodes + 4 * (2 * node + 1));
        fr_copy(s[2], nodes + 4 * (2 * node + 2));
    }
    for (int r = 0; r < 3; r++) {  /* addi rows: (s_r, 0, s_r + rk_r, 0) */
        uint64_t a[4];
        or_fr_add(a, s[r], pc + 4 * r);
        MK_ROW(r, s[r], zero, a, zero);
        fr_copy(s[r], a);
    }
    for (int k = 0; k < MK_ROUNDS; k++) {
        int full = k < 4 || k >= MK_ROUNDS - 4;
        mk_pow5(e[0], s[0]);
        if (full) { mk_pow5(e[1], s[1]); mk_pow5(e[2], s[2]); }
        else { fr_copy(e[1], s[1]); fr_copy(e[2], s[2]); }
        for (int j = 0; j < 3; j++) {
            or_fr_mul(o[j], pc + 4 * (MK_NRK + 3 * j), e[0]);
            or_fr_mul(t, pc + 4 * (MK_NRK + 3 * j + 1), e[1]); or_fr_add(o[j], o[j], t);
            or_fr_mul(t, pc + 4 * (MK_NRK + 3 * j + 2), e[2]); or_fr_add(o[j], o[j], t);
            if (k < MK_ROUNDS - 1) or_fr_add(o[j], o[j], pc + 4 * (3 * k + 3 + j));
            MK_ROW(3 + 3 * k + j, s[0], s[1], o[j], s[2]);
        }
        memcpy(s, o, sizeof s);
    }
    MK_ROW(MK_ROWS - 1, s[1], s[1], zero, zero);  /* assert_equal(node, S_62,1) */
    fr_copy(nodes + 4 * node, s[1]);
#undef MK_ROW
}

/* selectors (q_l q_r q_o q_4 q_c q_hl q_hr q_h4 q_arith) and the copy
 * permutation's next slot (row, wire) for every wire of row i */
static void mk_layout_row(int H, uint64_t i, const uint64_t *pc, const uint64_t M1[4], const uint64_t *sel[9],
                          uint64_t nr[4], int nw[4]) {
    static const uint64_t Z[4] = {0, 0, 0, 0};
    const uint64_t NH = (1ULL << (H - 1)) - 1, root_row = MK_FIRST + MK_ROWS * NH;
    for (int q = 0; q < 9; q++) sel[q] = Z;
    for (int k = 0; k < 4; k++) nr[k] = i, nw[k] = k;
    enum { WL, WR, WO, W4 };
    const int win[3] = {WL, WR, W4};
#define TO(wire, r, w2) (nr[wire] = (r), nw[wire] = (w2))
    if (i == 0) {
        sel[0] = OR_FR_ONE, sel[8] = OR_FR_ONE;
        TO(WL, 0, WR), TO(WR, 0, WO), TO(WO, 0, W4), TO(W4, 3, WO);
    } else if (i == 2) {
        TO(WL, 3, WL), TO(WR, 3, WR);
    } else if (i == 3) {
        TO(WL, 2, WL), TO(WR, 2, WR), TO(WO, 3, W4), TO(W4, MK_FIRST, WR);
    } else if (i >= MK_FIRST && i < root_row) {
        const uint64_t p = (i - MK_FIRST) / MK_ROWS, hb = MK_FIRST + MK_ROWS * p;
        const int r = (int)(i - hb);
        const uint64_t node = mk_node_of(p, H);
        const int leaf_parent = node >= (1ULL << (H - 2)) - 1;
        if (r < 3) {
            sel[0] = OR_FR_ONE, sel[2] = M1, sel[4] = pc + 4 * r, sel[8] = OR_FR_ONE;
            if (r > 0 && !leaf_parent) {
                const uint64_t c = 2 * node + r;
                TO(WL, MK_FIRST + MK_ROWS * mk_hash_pos(c, H) + MK_ROWS - 1, WL);
            }
            TO(WR, i, W4);
            TO(W4, r < 2 ? i + 1 : hb + MK_ROWS - 1, r < 2 ? WR : WO);
            TO(WO, hb + 3, win[r]);
        } else if (r < MK_ROWS - 1) {
            const int k = (r - 3) / 3, j = (r - 3) % 3;
            const int full = k < 4 || k >= MK_ROUNDS - 4;
            sel[5] = pc + 4 * (MK_NRK + 3 * j);
            if (full) sel[6] = pc + 4 * (MK_NRK + 3 * j + 1), sel[7] = pc + 4 * (MK_NRK + 3 * j + 2);
            else sel[1] = pc + 4 * (MK_NRK + 3 * j + 1), sel[3] = pc + 4 * (MK_NRK + 3 * j + 2);
            if (k < MK_ROUNDS - 1) sel[4] = pc + 4 * (3 * k + 3 + j);
            sel[2] = M1, sel[8] = OR_FR_ONE;
            for (int x = 0; x < 3; x++) {
                const uint64_t producer = k == 0 ? hb + x : hb + 3 + 3 * (k - 1) + x;
                if (j < 2) TO(win[x], i + 1, win[x]);
                else TO(win[x], producer, WO);
            }
            if (k < MK_ROUNDS - 1) TO(WO, hb + 3 + 3 * (k + 1), win[j]);
            else if (j == 1) TO(WO, hb + MK_ROWS - 1, WR);
        } else {
            sel[0] = OR_FR_ONE, sel[1] = M1, sel[8] = OR_FR_ONE;
            if (node == 0) {
                TO(WL, root_row, WL);
            } else {
                const uint64_t par = (node - 1) / 2;
                TO(WL, MK_FIRST + MK_ROWS * mk_hash_pos(par, H) + ((node & 1) ? 1 : 2), WL);
            }
            TO(WR, hb + 3 + 3 * (MK_ROUNDS - 1) + 1, WO);
            TO(WO, i, W4);
            TO(W4, p + 1 < NH ? hb + MK_ROWS : root_row, WR);
        }
    } else if (i == root_row) {
        sel[0] = OR_FR_ONE, sel[2] = M1, sel[8] = OR_FR_ONE;
        TO(WL, root_row - 1, WL), TO(WR, i, WO), TO(WO, i, W4), TO(W4, 0, WL);
    }
#undef TO
}

/* pnp_synth_merkle on the CPU: w[4] (ng rows), sel[9] and sigma[4] (n rows),
 * nodes (2^(H-1) - 1), root_canon = the root (canonical).  Returns 0, or -1
 * when the circuit does not fit the domain. */
int or_synth_merkle(uint32_t height, const uint64_t *pc_mont, const uint64_t *leaves, const uint64_t *blind,
                    uint64_t *nodes, uint64_t *const w[4], uint64_t *const sel[9], uint64_t *const sigma[4],
                    uint64_t n, uint64_t root_canon[4]) {
    const int H = (int)height;
    const uint64_t ng = MK_FIRST + MK_ROWS * ((1ULL << (H - 1)) - 1) + 1;
    if (H < 2 || H > 20 || ng > n) return -1;
    uint32_t lg = 0;
    while ((1ULL << lg) < n) lg++;
    for (int j = 0; j < 4; j++) memset(w[j], 0, 32 * MK_FIRST);
    for (int r = 1; r <= 2; r++)
        for (int j = 0; j < 4; j++) fr_copy(w[j] + 4 * r, blind + 4 * (4 * (r - 1) + j));
    for (int j = 0; j < 2; j++) fr_copy(w[j] + 4 * 3, blind + 4 * (4 + j));
    for (int l = H - 2; l >= 0; l--) {
#pragma omp parallel for schedule(static)
        for (int64_t t = 0; t < (int64_t)(1ULL << l); t++)
            mk_hash_rows(H, (1ULL << l) - 1 + (uint64_t)t, pc_mont, leaves, nodes, w);
    }
    const uint64_t rr = ng - 1;
    for (int j = 1; j < 4; j++) memset(w[j] + 4 * rr, 0, 32);
    fr_copy(w[0] + 4 * rr, nodes);
    uint64_t omega[4], K[4][4];
    or_root_of_unity(omega, lg);
    fr_copy(K[0], OR_FR_ONE);
    or_fr_from_u64(K[1], 7);
    or_fr_from_u64(K[2], 13);
    or_fr_from_u64(K[3], 17);
    uint64_t M1[4];
    or_fr_neg(M1, OR_FR_ONE);
    /* omega^j for j < n as a table (sigma targets are arbitrary rows) */
    uint64_t *pw = (uint64_t *)malloc(32 * n);
    const int64_t CH = 4096;
#pragma omp parallel for schedule(static)
    for (int64_t c = 0; c < (int64_t)((n + CH - 1) / CH); c++) {
        uint64_t lo = (uint64_t)c * CH, hi = lo + CH < n ? lo + CH : n, x[4];
        or_fr_pow(x, omega, lo);
        for (uint64_t i = lo; i < hi; i++) { fr_copy(pw + 4 * i, x); or_fr_mul(x, x, omega); }
    }
#pragma omp parallel for schedule(static)
    for (int64_t ii = 0; ii < (int64_t)n; ii++) {
        const uint64_t i = (uint64_t)ii;
        const uint64_t *s9[9];
        uint64_t nr[4];
        int nw[4];
        mk_layout_row(H, i, pc_mont, M1, s9, nr, nw);
        for (int q = 0; q < 9; q++) fr_copy(sel[q] + 4 * i, s9[q]);
        for (int k = 0; k < 4; k++) or_fr_mul(sigma[k] + 4 * i, K[nw[k]], pw + 4 * nr[k]);
    }
    free(pw);
    or_fr_from_mont(root_canon, nodes);
    return 0;
}

/* k_coset_consts: x_i = 7 w_8n^i, vh_i = x_i^n - 1 (either may be NULL) */
void or_synth_coset_consts(uint64_t *vh, uint64_t *x, uint32_t lg) {
    uint64_t n = 1ULL << lg, N8 = n << 3, w8n[4], w8[4], g[4], gn[4], h[8][4];
    or_root_of_unity(w8n, lg + 3);
    or_root_of_unity(w8, 3);
    or_fr_from_u64(g, 7);
    or_fr_pow(gn, g, n);
    uint64_t p[4];
    fr_copy(p, gn);
    for (int k = 0; k < 8; k++) {
        or_fr_sub(h[k], p, OR_FR_ONE);
        or_fr_mul(p, p, w8);
    }
    const int64_t CH = 4096;
#pragma omp parallel for schedule(static)
    for (int64_t c = 0; c < (int64_t)((N8 + CH - 1) / CH); c++) {
        uint64_t lo = (uint64_t)c * CH, hi = lo + CH < N8 ? lo + CH : N8, xi[4];
        or_fr_pow(xi, w8n, lo);
        or_fr_mul(xi, xi, g);
        for (uint64_t i = lo; i < hi; i++) {
            if (x) fr_copy(x + 4 * i, xi);
            if (vh) fr_copy(vh + 4 * i, h[i & 7]);
            or_fr_mul(xi, xi, w8n);
        }
    }
}
