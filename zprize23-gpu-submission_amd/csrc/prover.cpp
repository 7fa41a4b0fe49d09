// prover.cpp — gen_proof orchestration on one MI355X.
//
// Protocol order and transcript labels follow the reference's prove()
// (lib/PLONK/src/gen_proof.cuh:10-489); the semantics are the ZK-Garage
// prover's (prover.rs:171-660), which the GPU path reproduces on its own
// circuit class (the Merkle circuit: no custom gates, no lookup tables, one
// public input) and abandons outside it (combine_split
// skipped, empty q_m / custom-selector / q_lookup coefficients, the 8-byte
// t_next / h1_next shift — proofs its verifier rejects).  Here, for any
// circuit: h1 / h2 from combine_split (lookup.hip), z2 with the true next
// row, the range / logic / fixed-base / curve-add widgets in the quotient
// (k_widgets) and the linearisation, q_m and q_lookup terms, and any number
// of public inputs (pnp_prove_ex).  On the Merkle class every extra term is
// zero and is skipped without a launch.
//
// What differs is HOW it runs on MI355X:
//   * the prover key and SRS are HBM-resident (pnp_load_*), no per-proof H2D
//     copies (the reference re-copies ~23 GB per proof, gen_proof.cuh:64-78,
//     166-180, quotient.cu:201-367);
//   * one stream, buffers sized once and reused (no per-op allocation);
//   * fused passes (protocol.hip) instead of ~100 single-op launches;
//   * MSMs of polynomials that are identically zero (h1, h2, and f / table
//     when the lookup tables are empty) are not launched: their commitment is
//     the point at infinity, exactly what the MSM would return;
//   * the 14 commitments in the openings whose values never reach the proof
//     (gen_proof.cuh:421, 450: aw/saw commits only feed empty randomness) are
//     not computed; z_comm is the z commitment (saw_commits[0] == commit(z)).
#include <chrono>
#include <string.h>
#include "context.h"
#include "protocol.h"
#include "transcript.h"
#include "widgets.cuh"
#include <algorithm>

namespace pnp {

Fr fr_from_u64(uint64_t x) {
    Fr r = Fr::zero();
    r.v[0] = (uint32_t)x;
    r.v[1] = (uint32_t)(x >> 32);
    return to_mont(r);
}

Fr root_of_unity(uint32_t lg) {
    const uint64_t root32[4] = {13381757501831005802ULL, 6564924994866501612ULL,
                                789602057691799140ULL, 6625830629041353339ULL};
    return pow_u64(from_u64_limbs<FrP>(root32), 1ULL << (32 - lg));
}

namespace {

struct Timer {
    pnp_ctx *ctx;
    std::chrono::steady_clock::time_point t0;
    explicit Timer(pnp_ctx *c) : ctx(c), t0(std::chrono::steady_clock::now()) { ctx->stages.clear(); }
    void mark(const char *name) {
        PNP_HIP(hipStreamSynchronize(ctx->stream));
        auto t1 = std::chrono::steady_clock::now();
        ctx->stages.emplace_back(name, std::chrono::duration<double, std::milli>(t1 - t0).count());
        t0 = t1;
    }
};

void append_comm(Transcript &t, const char *label, const CommitmentC &c) {
    t.append_point(label, c.x, c.y);
}

void set_infinity(CommitmentC *c) {
    memset(c, 0, sizeof *c);
    to_u64_limbs(Fq::one(), c->y);
}

void store_fr_host(uint64_t out[4], const Fr &a) { to_u64_limbs(a, out); }

// k words from every rank (rank-major), one tagged all-gather
std::vector<uint64_t> shard_allgather(pnp_ctx *ctx, const uint64_t *mine, int k, uint64_t tag) {
    return rank_allgather(ctx->msm, ctx->stream, mine, k, tag);
}

// In place p_k <- p_k / (X - z_k) (kzg10.cu:87-99) for the K polynomials of
// round 6, where this rank holds the coefficient range [a, a + len) of each.
// Quotient coefficient q_i = sum_(k > i) p_k z^(k-i-1) = (division of the
// local slice) + z^(a+len-1-i) C with C = sum_(k >= a+len) p_k z^(k-a-len):
// every rank shares the value E_r of its slice at z, C follows from the E of
// the ranks above — both polynomials' values in ONE all-gather.
void div_linear_range(pnp_ctx *ctx, uint64_t *const *d, const Fr *z, int K, uint64_t len, bool dist) {
    hipStream_t s = ctx->stream;
    if (!dist) {
        k_poly_div_linear_batch(d, z, K, len, ctx->scratch_a, s);  // one chain of launches for all K
        return;
    }
    const int world = ctx->msm.world, rank = ctx->msm.rank;
    std::vector<uint64_t> mine(4 * K);
    std::vector<Fr> e(K);
    std::vector<EvalSet> sets(K);
    for (int k = 0; k < K; k++) sets[k] = {d + k, 1, z[k], &e[k]};
    k_poly_eval_sets(sets.data(), K, len, ctx->scratch_a, s);
    for (int k = 0; k < K; k++) to_u64_limbs(e[k], &mine[4 * k]);
    std::vector<uint64_t> all = shard_allgather(ctx, mine.data(), 4 * K, PNP_EX_TAG_DIV_CARRY);
    const uint64_t n = len * world;  // equal ranges (world divides 8 and n)
    k_poly_div_linear_batch(d, z, K, len, ctx->scratch_a, s);
    for (int k = 0; k < K; k++) {
        Fr c = Fr::zero();
        const Fr zl = pow_u64(z[k], n / world);
        for (int r = world - 1; r > rank; r--) c = c * zl + from_u64_limbs<FrP>(&all[4 * (K * r + k)]);
        if (rank < world - 1) k_add_powers(d[k], len, c, z[k], s);
    }
}

}  // namespace

int prove_impl(pnp_ctx *ctx, const CircuitC *cs, int device_ptrs, ProofC *out, const ProveOpts *opt) {
    if (!ctx->pk_loaded || !ctx->ck_loaded) {
        set_error("prover key / commit key not loaded");
        return PNP_E_NOKEY;
    }
    memset(out, 0, sizeof *out);
    hipStream_t s = ctx->stream;
    PNP_HIP(hipSetDevice(ctx->device));
    uint64_t bound = cs->n > cs->lookup_len ? cs->n : cs->lookup_len;
    uint64_t n = 1;
    uint32_t lg = 0;
    while (n < bound) { n <<= 1; lg++; }
    if (n != ctx->pk_n) {
        set_error("circuit domain %llu != prover key domain %llu", (unsigned long long)n,
                  (unsigned long long)ctx->pk_n);
        return PNP_E_ARG;
    }
    if (ctx->ck_points < n) {
        set_error("commit key has %llu points, need %llu", (unsigned long long)ctx->ck_points,
                  (unsigned long long)n);
        return PNP_E_ARG;
    }
    // public inputs: v1 = the circuit's one (pi, intended_pi_pos), appended as
    // the reference GPU path does (transcript.cuh:39-44); v2 = a PublicInputs
    // map (pi.rs:16-86): BTreeMap order, zero values dropped
    std::vector<uint64_t> pi_pos;
    std::vector<Fr> pi_val;  // Montgomery
    if (!opt) {
        if (cs->intended_pi_pos >= n || !cs->pi) {
            set_error("public input position out of range");
            return PNP_E_ARG;
        }
        pi_pos.push_back(cs->intended_pi_pos);
        pi_val.push_back(to_mont(from_u64_limbs<FrP>(cs->pi)));
    } else {
        std::vector<std::pair<uint64_t, Fr>> v;
        for (uint64_t k = 0; k < opt->n_pi; k++) {
            if (opt->pi_pos[k] >= n) {
                set_error("public input position %llu out of range", (unsigned long long)opt->pi_pos[k]);
                return PNP_E_ARG;
            }
            v.emplace_back(opt->pi_pos[k], to_mont(from_u64_limbs<FrP>(opt->pi_canon + 4 * k)));
        }
        std::sort(v.begin(), v.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
        for (size_t k = 0; k < v.size(); k++) {
            if (k && v[k].first == v[k - 1].first) {
                set_error("public input position %llu given twice", (unsigned long long)v[k].first);
                return PNP_E_ARG;
            }
            if (v[k].second.is_zero()) continue;
            pi_pos.push_back(v[k].first);
            pi_val.push_back(v[k].second);
        }
    }
    // Deferred tables (context.h): a proof that finds the optional tables
    // missing goes without them.  One GPU: on by default, the tables are only
    // built in the background, started when such a proof returns; several
    // ranks: off by default, the context's first proof only (every rank: the
    // same call sequence; hbm_budget checks the ranks agree)
    if (ctx->defer_tables < 0) ctx->defer_tables = ctx->msm.world <= 1 ? 1 : 0;
    const bool bg_mode = ctx->msm.world <= 1 && tables_bg_enabled();
    ctx->defer_now = ctx->defer_tables == 1 && (bg_mode || ctx->proofs_started == 0);
    ctx->proofs_started++;
    ctx->tables_wanted = false;
    struct DeferScope {  // the deferral is this proof's only, on every exit
        pnp_ctx *c;
        ~DeferScope() { c->defer_now = false; }
    } defer_scope{ctx};
    if (!ctx->hbm_checked) {  // the first proof after a key load: the HBM budget (every rank)
        hbm_budget(ctx);
        ctx->hbm_checked = true;
    }
    ctx->msm.batch_seq = 0;  // the fixed-slot exchange keys its capacities by batch ordinal
    const uint64_t N8 = 8 * n, ng = cs->n;
    const ProverKeyC &pk = ctx->pk_dev;
    Timer tm(ctx);
    auto &nt = ctx->ntt;
    // The proof's algorithmic HBM bytes (the whole-proof GB/s
    // beside the wall-clock): every op below credits its minimal reads and
    // writes in Fr elements (32 B); the MSMs credit their scalars and the
    // accumulation its device-counted entries in msm.hip (bench.py adds them
    // up; DESIGN.md 5 states the tally)
    auto alg = [&](double elems) { ctx->ktimer.credit("proof_alg_bytes", 32.0 * elems); };
    k_proof_marker(s);
    // the twiddle / twist tables are built lazily; build them here, on the main
    // stream, so the side-stream LDEs (after fork()) and the main-stream LDEs
    // both read finished tables
    ntt_warm(nt, lg, s);
    // round-4 distribution (pnp_set_exchange_a2a, fixed at key load): this
    // rank's coset blocks [mb0, mb0 + nb) and coefficient range [q0, q0 + len)
    const int world = ctx->msm.world;
    if (ctx->pk_blk_world != world || ctx->pk_blk_rank != ctx->msm.rank) {
        set_error("sharding changed after pnp_load_prover_key");
        return PNP_E_ARG;
    }
    const int mb0 = ctx->pk_mb0, nb = ctx->pk_nb;
    const bool dist = nb < 8;
    const uint64_t NB = (uint64_t)nb * n;
    uint64_t q0 = 0, q1 = n;
    if (dist) msm_point_range(n, ctx->msm.rank, world, q0, q1);
    const uint64_t len = q1 - q0;
    // The round-4 coset LDEs of the wires and of z depend on no challenge:
    // they run on a low-priority side stream beside the round-1 / round-3
    // MSMs, whose sort, merge and tree phases leave most SIMDs idle, and the
    // quotient waits for them (PNP_NO_OVERLAP=1: in round 4, as before).
    static const bool overlap = getenv("PNP_NO_OVERLAP") == nullptr;
    hipStream_t s_lo = overlap ? ctx->side_stream() : s;
    // Round 4 on one GPU runs on the first 6 coset blocks, not all 8: the
    // quotient of a satisfying circuit has degree < 6n (the largest term,
    // q_arith q_hl a^5, has degree < 7n; the reference's t_7, t_8 are zero),
    // so its values on 6n points of the coset already determine it — 25% fewer
    // LDE transforms, quotient points and inverse transforms.  Round 5 checks
    // the quotient identity at the challenge z (lin(z) = -r_0, the verifier's
    // equation); a circuit the witness does not satisfy fails it and round 4
    // is redone on all 8 blocks, exactly the reference's computation.
    // (PNP_QUOT_BLOCKS = 6 .. 8; distributed round 4 keeps its 8 / world
    // blocks per rank.)
    static const int quot_blocks = [] {
        const char *e = getenv("PNP_QUOT_BLOCKS");
        int v = e ? atoi(e) : 6;
        return v < 6 ? 6 : v > 8 ? 8 : v;
    }();
    int nbq = dist ? nb : quot_blocks;  // blocks this round-4 attempt covers
    // The quotient of the common case (no custom gates, no lookup, the
    // standard coset: the Merkle circuit) runs in radix 2^29 (protocol.h
    // k_quotient29): its wire, z (and multi-PI) LDEs are taken in the 2^261
    // form (the scaled twist, free) and the key arrays it reads are the
    // 2^261-form copies made at key load; any other key keeps k_quotient_
    // (PNP_QUOT29=0: every key)
    const bool q29 = ctx->pk_q29;
    auto lde_on = [&](hipStream_t st, const uint64_t *coeffs, uint64_t *dst, bool f29) {
        lde_blocks(nt, coeffs, dst, lg, mb0, nbq, st, f29);
    };
    auto fork = [&]() {
        if (!overlap) return;
        PNP_HIP(hipEventRecord(ctx->ev_fork, s));
        PNP_HIP(hipStreamWaitEvent(s_lo, ctx->ev_fork, 0));
    };

    // ---------------- inputs: padded witness evaluations (pad_poly)
    uint64_t *wsc[4], *wpoly[4];
    const uint64_t *wsrc[4] = {cs->w_l, cs->w_r, cs->w_o, cs->w_4};
    std::vector<H2D> up;  // a host witness: staged uploads (abi.cpp h2d_batch)
    for (int j = 0; j < 4; j++) {
        wsc[j] = ctx->buf("wsc" + std::to_string(j), n);
        wpoly[j] = ctx->buf("wpoly" + std::to_string(j), n);
        if (device_ptrs) PNP_HIP(hipMemcpyAsync(wsc[j], wsrc[j], 32 * ng, hipMemcpyDeviceToDevice, s));
        else up.push_back({wsc[j], wsrc[j], 32 * ng});
        if (n > ng) PNP_HIP(hipMemsetAsync(wsc[j] + 4 * ng, 0, 32 * (n - ng), s));
    }
    uint64_t *qlk = ctx->buf("qlk", n);
    if (device_ptrs) PNP_HIP(hipMemcpyAsync(qlk, cs->q_lookup, 32 * ng, hipMemcpyDeviceToDevice, s));
    else up.push_back({qlk, cs->q_lookup, 32 * ng});
    if (!up.empty()) h2d_batch(ctx, up);
    alg(4.0 * (2 * ng + (n - ng)) + 2.0 * ng);
    tm.mark("inputs");

    Transcript tr(opt ? opt->label : "Merkle tree");
    if (!opt) {
        tr.append_pi("pi", cs->pi, cs->intended_pi_pos);
    } else {
        std::vector<uint64_t> canon(4 * pi_val.size());
        for (size_t k = 0; k < pi_val.size(); k++) to_u64_limbs(from_mont(pi_val[k]), &canon[4 * k]);
        tr.append_pis("pi", pi_pos.size(), pi_pos.data(), canon.data());
    }

    // ---------------- round 1: witness polynomials (gen_proof.cuh:25-50)
    // With the Lagrange-basis key the commitments are taken from the padded
    // evaluations (the same points; zero rows drop out of the MSM,
    // lagrange.hip), and the coefficients feed only the round-4 LDEs and
    // round 5: the wires' iNTTs move to the side stream with the LDEs, off
    // the commitments' path.
    const bool lag = lagrange_table(ctx, n) != nullptr;
    uint64_t *w8buf[4];
    for (int j = 0; j < 4; j++) w8buf[j] = ctx->buf("w8_" + std::to_string(j), NB);
    CommitmentC *wc[4] = {&out->a_comm, &out->b_comm, &out->c_comm, &out->d_comm};
    if (lag) {
        fork();
        for (int j = 0; j < 4; j++) ntt_run(nt, wpoly[j], lg, true, false, s_lo, wsc[j]);
        for (int j = 0; j < 4; j++) lde_on(s_lo, wpoly[j], w8buf[j], q29);
        if (overlap) PNP_HIP(hipEventRecord(ctx->ev_w8, s_lo));
        alg(4.0 * 2 * n + 4.0 * (1 + nbq) * n);  // 4 iNTTs, 4 LDEs onto nbq blocks
        tm.mark("r1_intt");
        // over the copy-constraint groups when the key has them and the
        // witness keeps them (wires.hip), else row by row
        const uint64_t *sc[4] = {wsc[0], wsc[1], wsc[2], wsc[3]};
        if (commit_wires_grouped(ctx, sc, n, wc)) alg(4.0 * n * 72 / 32);  // row, group, representative
        else commit_evals_batch(ctx, sc, 4, n, wc);
    } else {
        for (int j = 0; j < 4; j++) ntt_run(nt, wpoly[j], lg, true, false, s, wsc[j]);
        alg(4.0 * 2 * n + 4.0 * (1 + nbq) * n);
        tm.mark("r1_intt");
        fork();
        for (int j = 0; j < 4; j++) lde_on(s_lo, wpoly[j], w8buf[j], q29);
        if (overlap) PNP_HIP(hipEventRecord(ctx->ev_w8, s_lo));
        const uint64_t *sc[4] = {wpoly[0], wpoly[1], wpoly[2], wpoly[3]};
        commit_affine_batch(ctx, sc, 4, n, wc);
    }
    append_comm(tr, "w_l", *wc[0]);
    append_comm(tr, "w_r", *wc[1]);
    append_comm(tr, "w_o", *wc[2]);
    append_comm(tr, "w_4", *wc[3]);
    tm.mark("r1_commit");

    // ---------------- round 2: lookup (gen_proof.cuh:52-125)
    Fr zeta = tr.challenge_scalar("zeta");
    tr.append_scalar("zeta", zeta);
    uint64_t *tc = ctx->buf("tc", n), *table_poly = ctx->buf("table_poly", n);
    k_compress4(tc, pk.table1, pk.table2, pk.table3, pk.table4, zeta, n, s);
    const bool table_zero = !k_any_nonzero(tc, 4 * n, ctx->scratch_b, s);
    uint64_t *fc = ctx->buf("fc", n), *f_poly = ctx->buf("f_poly", n);
    const uint64_t *wconst[4] = {wsc[0], wsc[1], wsc[2], wsc[3]};
    k_query_f(fc, qlk, ng, wconst, tc, zeta, n, s);
    const bool f_zero = !k_any_nonzero(fc, 4 * n, ctx->scratch_b, s);
    alg(5.0 * n + n + ng + n + n);  // compress, its check, query (q_lookup in, f out), its check
    // (zero f / table: their polynomials are never read)
    if (!table_zero) ntt_run(nt, table_poly, lg, true, false, s, tc);
    if (!f_zero) ntt_run(nt, f_poly, lg, true, false, s, fc);
    // s = sorted concatenation of f and t, halves h1 / h2 (prover.rs:304-329).
    // f = t = 0 (the Merkle circuit): h1 = h2 = 0, commitments at infinity.
    // The f, h1, h2 MSMs are independent of the transcript in between, so
    // they run as one batch.
    const bool h_zero = f_zero && table_zero;
    uint64_t *h1 = ctx->buf("h1", n), *h2 = ctx->buf("h2", n);
    uint64_t *h1_poly = ctx->buf("h1_poly", n), *h2_poly = ctx->buf("h2_poly", n);
    {
        const uint64_t *sc[3];
        CommitmentC *oc[3];
        int nc = 0;
        if (f_zero) {
            set_infinity(&out->f_comm);
        } else {
            sc[nc] = f_poly;
            oc[nc++] = &out->f_comm;
        }
        if (h_zero) {
            PNP_HIP(hipMemsetAsync(h1, 0, 32 * n, s));
            PNP_HIP(hipMemsetAsync(h2, 0, 32 * n, s));
            alg(2.0 * n);
            set_infinity(&out->h_1_comm);
            set_infinity(&out->h_2_comm);
        } else {
            if (!combine_split(ctx, tc, fc, n, h1, h2, s)) {
                set_error("lookup: a query value is not in the lookup table (Error::ElementNotIndexed)");
                return PNP_E_ARG;
            }
            ntt_run(nt, h1_poly, lg, true, false, s, h1);
            ntt_run(nt, h2_poly, lg, true, false, s, h2);
            sc[nc] = h1_poly;
            oc[nc++] = &out->h_1_comm;
            sc[nc] = h2_poly;
            oc[nc++] = &out->h_2_comm;
        }
        if (nc) commit_affine_batch(ctx, sc, nc, n, oc);
    }
    append_comm(tr, "f", out->f_comm);
    append_comm(tr, "h1", out->h_1_comm);
    append_comm(tr, "h2", out->h_2_comm);
    tm.mark("r2_lookup");

    // ---------------- round 3: permutation (gen_proof.cuh:127-208)
    Fr beta = tr.challenge_scalar("beta");
    tr.append_scalar("beta", beta);
    Fr gamma = tr.challenge_scalar("gamma");
    tr.append_scalar("gamma", gamma);
    Fr delta = tr.challenge_scalar("delta");
    tr.append_scalar("delta", delta);
    Fr eps = tr.challenge_scalar("epsilon");
    tr.append_scalar("epsilon", eps);
    if (beta == gamma || beta == delta || beta == eps || gamma == delta || gamma == eps ||
        delta == eps) {
        set_error("challenges must be different");  // gen_proof.cuh:152-157 asserts
        return PNP_E_ARG;
    }
    PermArgs pa;
    const uint64_t *sigc[4] = {pk.left_sigma_coeffs, pk.right_sigma_coeffs, pk.out_sigma_coeffs,
                               pk.fourth_sigma_coeffs};
    (void)sigc;
    for (int j = 0; j < 4; j++) {
        pa.w[j] = wsc[j];
        pa.sigma[j] = ctx->pk_sigma_n[j].u64();  // NTT.forward(sigma_polys[j]), cached at key load
    }
    const uint64_t kv[4] = {1, 7, 13, 17};  // K1..K3 (permutation/constants.cu:3-15)
    for (int j = 0; j < 4; j++) pa.bk[j] = beta * fr_from_u64(kv[j]);
    pa.beta = beta;
    pa.gamma = gamma;
    pa.omega = root_of_unity(lg);
    pa.tw = ntt_twiddles(nt, lg, false, s);  // built by ntt_warm above
    uint64_t *num = ctx->buf("num", n), *den = ctx->buf("den", n);
    uint64_t *z_poly = ctx->buf("z_poly", n);
    k_perm_numden(num, den, pa, n, s);
    k_batch_inverse(den, n, ctx->scratch_a, s);
    k_mul_inplace(num, den, n, s);
    k_prefix_product(num, n, ctx->scratch_a, s);
    alg(10.0 * n + 2.0 * n + 3.0 * n + 2.0 * n);  // numerators / denominators, inverse, product, scan
    alg(2.0 * n + (1.0 + nbq) * n);               // z's iNTT and LDE
    uint64_t *z8 = ctx->buf("z8", NB);
    if (lag) {  // z from its evaluations; its iNTT joins its LDE on the side stream
        fork();
        ntt_run(nt, z_poly, lg, true, false, s_lo, num);
        lde_on(s_lo, z_poly, z8, q29);
        if (overlap) PNP_HIP(hipEventRecord(ctx->ev_z8, s_lo));
        tm.mark("r3_z");
        const uint64_t *sc[1] = {num};
        CommitmentC *oc[1] = {&out->z_comm};
        // z is constant over runs of rows sigma fixes (the padding): one
        // scalar per run (wires.hip), else row by row
        if (commit_z_grouped(ctx, num, n, &out->z_comm)) alg(1.0 * n * 72 / 32);
        else commit_evals_batch(ctx, sc, 1, n, oc);
    } else {
        ntt_run(nt, z_poly, lg, true, false, s, num);
        tm.mark("r3_z");
        fork();
        lde_on(s_lo, z_poly, z8, q29);
        if (overlap) PNP_HIP(hipEventRecord(ctx->ev_z8, s_lo));
        commit_affine(ctx, z_poly, n, &out->z_comm);
    }
    append_comm(tr, "z", out->z_comm);
    // lookup grand product (permutation/mod.rs:754-822)
    uint64_t *z2_poly = ctx->buf("z2_poly", n);
    // lookup-trivial case (f = t = h1 = h2 = 0): every ratio is
    // (1+d) e (e(1+d)) / (e(1+d))^2 = 1, so z2 = 1 and its coefficients are [1, 0, ...]
    const bool z2_one = h_zero;
    if (z2_one) {
        uint64_t one[4];
        to_u64_limbs(Fr::one(), one);
        PNP_HIP(hipMemsetAsync(z2_poly, 0, 32 * n, s));
        PNP_HIP(hipMemcpyAsync(z2_poly, one, 32, hipMemcpyHostToDevice, s));
        PNP_HIP(hipStreamSynchronize(s));
    } else {
        // num is rewritten: the side stream's z iNTT must have read it
        if (lag && overlap) PNP_HIP(hipStreamWaitEvent(s, ctx->ev_z8, 0));
        k_lookup_nd(num, den, fc, tc, h1, h2, delta, eps, n, s);
        k_batch_inverse(den, n, ctx->scratch_a, s);
        k_mul_inplace(num, den, n, s);
        k_prefix_product(num, n, ctx->scratch_a, s);
        ntt_run(nt, z2_poly, lg, true, false, s, num);
    }
    // z_2_comm is not appended to the transcript (gen_proof.cuh:200-205): its
    // MSM is batched with the quotient chunks in round 4
    // public input poly (pi.cu:11-15)
    // = iNTT of the evaluations v * e_pos, in closed form: v n^-1 w^(-pos j)
    const Fr n_inv = inverse(fr_from_u64(n));
    const bool closed = ctx->pk_std_coset;  // L1 (and one PI) on the coset in closed form
    const bool pi_closed = closed && pi_pos.size() == 1;
    uint64_t *pi_poly = nullptr;
    if (pi_pos.size() == 1 && !closed) {
        pi_poly = ctx->buf("pi_poly", n);
        Fr w_inv_pos = pow_u64(inverse(root_of_unity(lg)), pi_pos[0]);
        k_geometric(pi_poly, n, pi_val[0] * n_inv, w_inv_pos, s);
    } else if (pi_pos.size() > 1) {  // iNTT of the sparse evaluations (pi.rs:76-86)
        pi_poly = ctx->buf("pi_poly", n);
        PNP_HIP(hipMemsetAsync(pi_poly, 0, 32 * n, s));
        std::vector<uint64_t> limbs(4 * pi_val.size());
        for (size_t k = 0; k < pi_val.size(); k++) to_u64_limbs(pi_val[k], &limbs[4 * k]);
        for (size_t k = 0; k < pi_val.size(); k++)
            PNP_HIP(hipMemcpyAsync(pi_poly + 4 * pi_pos[k], &limbs[4 * k], 32, hipMemcpyHostToDevice, s));
        PNP_HIP(hipStreamSynchronize(s));
        ntt_run(nt, pi_poly, lg, true, false, s);
    }
    if (pi_closed && ctx->pk_pinv_pos != pi_pos[0]) {
        // 1 / (x_i - w^pos) on this rank's blocks, kept across proofs with the
        // same PI position
        ctx->pk_pinv_pos = ~0ULL;
        if (ctx->pk_pinv.bytes < 32 * NB) ctx->pk_pinv.alloc(32 * NB);
        Fr wpos = pow_u64(root_of_unity(lg), pi_pos[0]);
        k_affine(ctx->pk_pinv.u64(), ctx->blk("lin"), Fr::one(), neg(wpos), NB, s);
        k_batch_inverse(ctx->pk_pinv.u64(), NB, ctx->scratch_a, s);
        ctx->pk_pinv_pos = pi_pos[0];
    }
    tm.mark("r3_z2_pi");

    // ---------------- round 4: quotient (gen_proof.cuh:209-267, quotient.cu:142-376)
    // (a satisfying circuit: one pass over nbq blocks; see quot_blocks above)
    const Transcript tr3 = tr;  // before the round-4 challenges
    for (;;) {
        const uint64_t NBq = (uint64_t)nbq * n;
        Fr alpha = tr.challenge_scalar("alpha");
        tr.append_scalar("alpha", alpha);
        Fr range_c = tr.challenge_scalar("range separation challenge");
        tr.append_scalar("range seperation challenge", range_c);
        Fr logic_c = tr.challenge_scalar("logic separation challenge");
        tr.append_scalar("logic seperation challenge", logic_c);
        Fr fixed_c = tr.challenge_scalar("fixed base separation challenge");
        tr.append_scalar("fixed base separation challenge", fixed_c);
        Fr var_c = tr.challenge_scalar("variable base separation challenge");
        tr.append_scalar("variable base separation challenge", var_c);
        Fr lsep = tr.challenge_scalar("lookup separation challenge");
        tr.append_scalar("lookup separation challenge", lsep);

        QuotArgs q;
        // coset evaluations in block layout, this rank's blocks only
        auto lde = [&](const uint64_t *coeffs, uint64_t *dst) { lde_on(s, coeffs, dst, false); };
        for (int j = 0; j < 4; j++) q.w8[j] = w8buf[j];
        uint64_t *z28 = ctx->buf("z28", NB);
        q.z8 = z8;
        q.pi8 = nullptr;
        q.l18 = q.l1v = q.pinv = nullptr;
        if (closed) q.l1v = ctx->blk("l1v");
        if (pi_closed) {
            q.pinv = ctx->pk_pinv.u64();
            q.c_pi = pi_val[0] * pow_u64(root_of_unity(lg), pi_pos[0]) * n_inv;
        } else if (pi_poly) {
            uint64_t *pi8 = ctx->buf("pi8", NB);
            lde_on(s, pi_poly, pi8, q29);
            q.pi8 = pi8;
        }
        q.z28 = nullptr;  // z2 = 1: its quotient terms cancel (protocol.h)
        if (!z2_one) {
            lde(z2_poly, z28);
            q.z28 = z28;
        }
        q.f8 = q.t8 = nullptr;
        if (!f_zero) {
            uint64_t *f8 = ctx->buf("f8", NB);
            lde(f_poly, f8);
            q.f8 = f8;
        }
        if (!table_zero) {
            uint64_t *t8 = ctx->buf("t8", NB);
            lde(table_poly, t8);
            q.t8 = t8;
        }
        q.h18 = q.h28 = nullptr;  // h1 = h2 = 0
        if (!h_zero) {
            uint64_t *h18 = ctx->buf("h18", NB), *h28 = ctx->buf("h28", NB);
            lde(h1_poly, h18);
            lde(h2_poly, h28);
            q.h18 = h18;
            q.h28 = h28;
        }
        // compute_first_lagrange_poly_scaled(n, alpha^2) and (n, 1) (quotient.cu:3-8):
        // one LDE of L1 (coefficients n^-1, no iNTT); alpha^2 is applied in the kernel
        Fr alpha2 = alpha * alpha;
        if (!closed) {
            uint64_t *l1 = ctx->buf("l1", n), *l18 = ctx->buf("l18", NB);
            k_geometric(l1, n, n_inv, Fr::one(), s);
            lde(l1, l18);
            q.l18 = l18;
        }
        q.alpha2 = alpha2;
        // prover-key evaluations: block-layout copies made at key load
        q.q_m = ctx->blk("q_m");  // nullptr = zero selector
        q.q_l = ctx->blk("q_l");
        q.q_r = ctx->blk("q_r");
        q.q_o = ctx->blk("q_o");
        q.q_4 = ctx->blk("q_4");
        q.q_c = ctx->blk("q_c");
        q.q_hl = ctx->blk("q_hl");
        q.q_hr = ctx->blk("q_hr");
        q.q_h4 = ctx->blk("q_h4");
        q.q_arith = ctx->blk("q_arith");
        q.q_lookup = ctx->blk("q_lookup");
        q.sig[0] = ctx->blk("sig0");
        q.sig[1] = ctx->blk("sig1");
        q.sig[2] = ctx->blk("sig2");
        q.sig[3] = ctx->blk("sig3");
        q.lin = ctx->blk("lin");
        q.vh_inv = ctx->blk("vh_inv");  // v_h^-1, computed at key load
        q.n = n;
        q.lg_n = lg;
        q.alpha = alpha;
        q.beta = beta;
        q.gamma = gamma;
        q.delta = delta;
        q.eps = eps;
        q.zeta = zeta;
        q.lsep = lsep;
        // the kernel derives beta k_j from beta for k = 1, 7, 13, 17
        for (int j = 0; j < 4; j++) q.bk[j] = pa.bk[j];
        if (!(pa.bk[1] == beta * fr_from_u64(7) && pa.bk[2] == beta * fr_from_u64(13) &&
              pa.bk[3] == beta * fr_from_u64(17))) {
            set_error("quotient: unexpected permutation coset constants");
            return PNP_E_ARG;
        }
        q.opd = delta + Fr::one();
        q.eopd = eps * q.opd;
        q.sep2 = lsep * lsep;
        q.sep3 = q.sep2 * lsep;
        if (overlap) {  // the side-stream LDEs of the wires and z
            PNP_HIP(hipStreamWaitEvent(s, ctx->ev_w8, 0));
            PNP_HIP(hipStreamWaitEvent(s, ctx->ev_z8, 0));
        }
        tm.mark("r4_lde");
        uint64_t *t_blk = ctx->buf("t_blk", NB);
        hipEvent_t qe0 = nullptr;
        ctx->ktimer.begin("quotient", s, qe0);
        if (q29) {
            Quot29Args q2;
            for (int j = 0; j < 4; j++) q2.w8[j] = q.w8[j];
            q2.z8 = q.z8;
            q2.pi8 = q.pi8;
            q2.q_m = ctx->blk29("q_m");
            q2.q_l = ctx->blk29("q_l");
            q2.q_r = ctx->blk29("q_r");
            q2.q_o = ctx->blk29("q_o");
            q2.q_4 = ctx->blk29("q_4");
            q2.q_c = ctx->blk29("q_c");
            q2.q_hl = ctx->blk29("q_hl");
            q2.q_hr = ctx->blk29("q_hr");
            q2.q_h4 = ctx->blk29("q_h4");
            q2.q_arith = ctx->blk29("q_arith");
            for (int j = 0; j < 4; j++) q2.sig[j] = ctx->blk29(("sig" + std::to_string(j)).c_str());
            q2.lin = ctx->blk29("lin");
            q2.vh_inv = q.vh_inv;
            q2.l1v = q.l1v;
            q2.pinv = q.pinv;
            fr_to_r29_limbs(q.pinv ? q.c_pi : Fr::zero(), q2.c_pi);
            fr_to_r29_limbs(alpha, q2.alpha);
            fr_to_r29_limbs(alpha2, q2.alpha2);
            fr_to_r29_limbs(beta, q2.beta);
            fr_to_r29_limbs(gamma, q2.gamma);
            fr_to_r29_limbs(Fr::one(), q2.one);
            q2.n = n;
            q2.lg_n = lg;
            if (!q2.l1v || !q2.q_l || !q2.lin || !q2.sig[3]) {
                set_error("quotient29: key copies missing");
                return PNP_E_ARG;
            }
            k_quotient29(q2, NBq, t_blk, s);
            // VALU work for bench.py's roofline: Fr products per point on the
            // path this launch takes (protocol.hip k_quotient29_: 5 paired
            // products = 10, three fifth powers = 9, 14 more; + 2 with q_m, + 1
            // with the closed-form PI)
            ctx->ktimer.credit("quotient_points", (double)NBq);
            ctx->ktimer.credit("quotient_fr_products",
                               (double)NBq * (34 + (q2.q_m ? 2 : 0) + (q2.pinv ? 1 : 0)));
            // (the byte accounting below counts the arrays this kernel read)
            q.q_m = q2.q_m, q.q_l = q2.q_l, q.q_r = q2.q_r, q.q_o = q2.q_o, q.q_4 = q2.q_4, q.q_c = q2.q_c;
            q.q_hl = q2.q_hl, q.q_hr = q2.q_hr, q.q_h4 = q2.q_h4, q.q_arith = q2.q_arith, q.lin = q2.lin;
            for (int j = 0; j < 4; j++) q.sig[j] = q2.sig[j];
        } else {
            k_quotient(q, NBq, t_blk, s);
        }
        if (ctx->pk_custom_nz[0] || ctx->pk_custom_nz[1] || ctx->pk_custom_nz[2] || ctx->pk_custom_nz[3]) {
            WidgetArgs g;
            for (int j = 0; j < 4; j++) g.w8[j] = q.w8[j];
            g.q_l = q.q_l;
            g.q_r = q.q_r;
            g.q_c = q.q_c;
            g.vh_inv = q.vh_inv;
            g.sel[0] = ctx->blk("range");
            g.sel[1] = ctx->blk("logic");
            g.sel[2] = ctx->blk("fixed_add");
            g.sel[3] = ctx->blk("var_add");
            g.sep[0] = range_c;
            g.sep[1] = logic_c;
            g.sep[2] = fixed_c;
            g.sep[3] = var_c;
            g.n = n;
            g.lg_n = lg;
            k_widgets(g, NBq, t_blk, s);
        }
        {
            // algorithmic bytes: every coset array the kernel reads (nullptr = known
            // zero, not read) plus t, 32 B per point each
            const uint64_t *arrs[] = {q.w8[0], q.w8[1], q.w8[2], q.w8[3], q.q_m, q.q_l, q.q_r, q.q_o,
                                      q.q_4, q.q_c, q.q_hl, q.q_hr, q.q_h4, q.q_arith, q.pi8, q.lin,
                                      q.z8, q.sig[0], q.sig[1], q.sig[2], q.sig[3], q.f8,
                                      q.t8, q.h18, q.h28, q.q_lookup, q.z28, q.l18, q.vh_inv, q.l1v, q.pinv};
            int nread = 0;
            for (const uint64_t *a : arrs) nread += a != nullptr;
            ctx->ktimer.end("quotient", s, qe0, 32.0 * (double)NBq * (nread + 1));
            alg((double)NBq * (nread + 1));
        }
        tm.mark("r4_quotient");
        // Intt_coset of the coset values: per block an unscaled size-n inverse
        // transform and a twist, then per coefficient index an inverse DFT (8
        // blocks, ntt.hip t_combine) or Vandermonde solve (6 / 7 blocks,
        // t_combine_blocks) across the blocks -> the chunks t_1..t_8, here over
        // this rank's coefficient range [q0, q0 + len): t_poly[k len + u]; with
        // nbq < 8 blocks the chunks from t_(nbq+1) on are zero
        intt_blocks(nt, t_blk, lg, mb0, nbq, s);
        alg(2.0 * NBq + 2.0 * NBq);  // the block iNTTs and the combine
        uint64_t *t_poly = ctx->buf("t_poly", 8 * len);
        const int npieces = dist ? 8 : nbq;
        unsigned *t_nz = reinterpret_cast<unsigned *>(ctx->buf("t_nz", 1));  // bit k: chunk k != 0
        PNP_HIP(hipMemsetAsync(t_nz, 0, 4, s));
        if (!dist) {
            t_combine_blocks(nt, t_blk, nbq, t_poly, lg, t_nz, s);
        } else {
            // all-to-all: rank r' receives, from every rank, that rank's blocks
            // restricted to r''s coefficient range; slots arrive block-major
            const uint64_t slot = (uint64_t)nb * len * 32;
            if (!ctx->msm.alltoall || ctx->msm.a2a_bytes < 2 * slot * world) {
                set_error("round-4 all-to-all buffer missing or < %llu B",
                          (unsigned long long)(2 * slot * world));
                return PNP_E_ARG;
            }
            uint64_t *a2a = ctx->msm.a2a;
            for (int r = 0; r < world; r++) {
                uint64_t r0, r1;
                msm_point_range(n, r, world, r0, r1);
                for (int b = 0; b < nb; b++)
                    PNP_HIP(hipMemcpyAsync(a2a + 4 * ((uint64_t)(r * nb + b) * len), t_blk + 4 * ((uint64_t)b * n + r0),
                                           32 * len, hipMemcpyDeviceToDevice, s));
            }
            ex_fence(ctx->msm, s);
            int rc = ctx->msm.alltoall(ctx->msm.a2a_user, slot);
            if (rc != 0) {
                set_error("round-4 all-to-all callback failed (%d)", rc);
                return PNP_E_DEVICE;
            }
            t_combine(nt, a2a + 4 * (uint64_t)nb * len * world, len, q0, t_poly, lg, t_nz, s);
        }
        tm.mark("r4_intt8");
        CommitmentC *tcm[8] = {&out->t_1_comm, &out->t_2_comm, &out->t_3_comm, &out->t_4_comm,
                               &out->t_5_comm, &out->t_6_comm, &out->t_7_comm, &out->t_8_comm};
        {
            // chunks that are identically zero (t_7, t_8 for a satisfying circuit:
            // deg t < 6n) commit to the point at infinity without an MSM
            const uint64_t *sc[9];
            CommitmentC *oc[9];
            int nc = 0;
            uint64_t nz[8];
            {
                unsigned bits = 0;  // flagged by the combine kernel as it wrote the chunks
                PNP_HIP(hipMemcpyAsync(&bits, t_nz, 4, hipMemcpyDeviceToHost, s));
                PNP_HIP(hipStreamSynchronize(s));
                for (int k = 0; k < 8; k++) nz[k] = k < npieces && ((bits >> k) & 1);
            }
            if (dist) {  // a chunk is zero when it is zero on every rank (own slot included)
                std::vector<uint64_t> all = shard_allgather(ctx, nz, 8, PNP_EX_TAG_T_FLAGS);
                for (int k = 0; k < 8; k++) {
                    nz[k] = 0;
                    for (int r = 0; r < world; r++) nz[k] |= all[8 * r + k];
                }
            }
            for (int k = 0; k < 8; k++) {
                if (!nz[k]) {
                    set_infinity(tcm[k]);
                    continue;
                }
                sc[nc] = t_poly + 4 * (uint64_t)k * len;
                oc[nc++] = tcm[k];
            }
            if (z2_one) {
                // commit([1, 0, ...]) = 1 * powers_of_g[0], already affine
                uint64_t g0[12];
                PNP_HIP(hipMemcpyAsync(g0, ctx->ck_dev, sizeof g0, hipMemcpyDeviceToHost, s));
                PNP_HIP(hipStreamSynchronize(s));
                memcpy(out->z_2_comm.x, g0, 48);
                memcpy(out->z_2_comm.y, g0 + 6, 48);
            } else if (dist) {
                commit_affine(ctx, z2_poly, n, &out->z_2_comm);
            } else {
                sc[nc] = z2_poly;
                oc[nc++] = &out->z_2_comm;
            }
            // distributed: the chunks hold this rank's coefficient range only,
            // exactly the point range of its MSM share
            commit_affine_batch(ctx, sc, nc, n, oc, dist);
        }
        const char *tl[8] = {"t_1", "t_2", "t_3", "t_4", "t_5", "t_6", "t_7", "t_8"};
        for (int k = 0; k < 8; k++) append_comm(tr, tl[k], *tcm[k]);
        tm.mark("r4_commit");
        ctx->ktimer.collect();  // the quotient's events (the commitments' read-back drained the stream)

        // ---------------- round 5: linearisation (linearisation.cu:73-306)
        Fr zc = tr.challenge_scalar("z");
        tr.append_scalar("z", zc);
        Fr omega = root_of_unity(lg);
        Fr zw = zc * omega;
        Fr vh = pow_u64(zc, n) - Fr::one();
        Fr zn = vh + Fr::one();
        Fr l1e = vh * inverse(fr_from_u64(n) * (zc - Fr::one()));
        ProofEvaluationsC *ev = &out->evaluations;
        {
            // evaluations at z
            // (distributed: every rank evaluates its coefficient range [q0, q0 + len)
            // of these replicated polynomials, scales by x^q0, and one all-gather
            // of the 18 partial values sums them)
            const uint64_t eo = 4 * q0;
            const uint64_t *pz[12] = {wpoly[0] + eo, wpoly[1] + eo, wpoly[2] + eo, wpoly[3] + eo,
                                      pk.left_sigma_coeffs + eo, pk.right_sigma_coeffs + eo,
                                      pk.out_sigma_coeffs + eo, pk.q_arith_coeffs + eo, pk.q_c_coeffs + eo,
                                      pk.q_l_coeffs + eo, pk.q_r_coeffs + eo, pk.q_hl_coeffs + eo};
            Fr rz[12];
            const uint64_t *pz2[2] = {pk.q_hr_coeffs + eo, pk.q_h4_coeffs + eo};
            Fr rz2[2];
            // evaluations at z * omega
            const uint64_t *pw[4] = {z_poly + eo, wpoly[0] + eo, wpoly[1] + eo, wpoly[3] + eo};
            Fr rw[4];
            const EvalSet sets[3] = {{pz, 12, zc, rz}, {pz2, 2, zc, rz2}, {pw, 4, zw, rw}};
            k_poly_eval_sets(sets, 3, len, ctx->scratch_a, s);  // one host round trip
            alg(18.0 * len);
            if (dist) {
                Fr *vals[18];
                for (int k = 0; k < 12; k++) vals[k] = &rz[k];
                vals[12] = &rz2[0], vals[13] = &rz2[1];
                for (int k = 0; k < 4; k++) vals[14 + k] = &rw[k];
                const Fr sz = pow_u64(zc, q0), sw = pow_u64(zw, q0);
                uint64_t mine[4 * 18];
                for (int k = 0; k < 18; k++) to_u64_limbs(*vals[k] * (k < 14 ? sz : sw), mine + 4 * k);
                std::vector<uint64_t> all = shard_allgather(ctx, mine, 4 * 18, PNP_EX_TAG_EVALS);
                for (int k = 0; k < 18; k++) {
                    Fr acc = Fr::zero();
                    for (int r = 0; r < world; r++) acc += from_u64_limbs<FrP>(&all[4 * (18 * r + k)]);
                    *vals[k] = acc;
                }
            }
            Fr z2n = Fr::one();
            if (!z2_one) k_poly_eval(z2_poly, n, zw, ctx->scratch_a, &z2n, s);
            Fr f_eval = Fr::zero(), t_eval = Fr::zero(), t_next = Fr::zero();
            Fr ql_eval = Fr::zero(), h1_eval = Fr::zero(), h1_next = Fr::zero(), h2_eval = Fr::zero();
            if (!ctx->pk_qlookup_zero) k_poly_eval(pk.q_lookup_coeffs, n, zc, ctx->scratch_a, &ql_eval, s);
            if (!h_zero) {
                k_poly_eval(h1_poly, n, zc, ctx->scratch_a, &h1_eval, s);
                k_poly_eval(h1_poly, n, zw, ctx->scratch_a, &h1_next, s);
                k_poly_eval(h2_poly, n, zc, ctx->scratch_a, &h2_eval, s);
            }
            if (!f_zero) k_poly_eval(f_poly, n, zc, ctx->scratch_a, &f_eval, s);
            if (!table_zero) {
                k_poly_eval(table_poly, n, zc, ctx->scratch_a, &t_eval, s);
                k_poly_eval(table_poly, n, zw, ctx->scratch_a, &t_next, s);
            }
            store_fr_host(ev->wire_evals.a_eval, rz[0]);
            store_fr_host(ev->wire_evals.b_eval, rz[1]);
            store_fr_host(ev->wire_evals.c_eval, rz[2]);
            store_fr_host(ev->wire_evals.d_eval, rz[3]);
            store_fr_host(ev->perm_evals.left_sigma_eval, rz[4]);
            store_fr_host(ev->perm_evals.right_sigma_eval, rz[5]);
            store_fr_host(ev->perm_evals.out_sigma_eval, rz[6]);
            store_fr_host(ev->perm_evals.permutation_eval, rw[0]);
            CustomEvaluationsC *cu = &ev->custom_evals;
            store_fr_host(cu->q_arith_eval, rz[7]);
            store_fr_host(cu->q_c_eval, rz[8]);
            store_fr_host(cu->q_l_eval, rz[9]);
            store_fr_host(cu->q_r_eval, rz[10]);
            store_fr_host(cu->q_hl_eval, rz[11]);
            store_fr_host(cu->q_hr_eval, rz2[0]);
            store_fr_host(cu->q_h4_eval, rz2[1]);
            store_fr_host(cu->a_next_eval, rw[1]);
            store_fr_host(cu->b_next_eval, rw[2]);
            store_fr_host(cu->d_next_eval, rw[3]);
            LookupEvaluationsC *lk = &ev->lookup_evals;
            store_fr_host(lk->q_lookup_eval, ql_eval);
            store_fr_host(lk->h1_eval, h1_eval);
            store_fr_host(lk->h1_next_eval, h1_next);
            store_fr_host(lk->h2_eval, h2_eval);
            store_fr_host(lk->z2_next_eval, z2n);
            store_fr_host(lk->f_eval, f_eval);
            store_fr_host(lk->table_eval, t_eval);
            store_fr_host(lk->table_next_eval, t_next);
        }
        tm.mark("r5_evals");
        auto ld = [](const uint64_t *p) { return from_u64_limbs<FrP>(p); };
        const Fr ae = ld(ev->wire_evals.a_eval), be = ld(ev->wire_evals.b_eval),
                 ce = ld(ev->wire_evals.c_eval), de = ld(ev->wire_evals.d_eval);
        const Fr qae = ld(ev->custom_evals.q_arith_eval);
        LinArgs la;
        la.k = 0;
        // over this rank's coefficient range (replicated polynomials offset by q0)
        auto push_local = [&](const uint64_t *p, const Fr &sc) {
            la.p[la.k] = p;
            la.s[la.k] = sc;
            la.k++;
        };
        auto push = [&](const uint64_t *p, const Fr &sc) { push_local(p + 4 * q0, sc); };
        auto p5 = [](const Fr &x) { Fr x2 = x * x; return x2 * x2 * x; };
        // arithmetic (widget/arithmetic.rs:82-100)
        if (!ctx->pk_qm_zero) push(pk.q_m_coeffs, ae * be * qae);
        push(pk.q_l_coeffs, ae * qae);
        push(pk.q_r_coeffs, be * qae);
        push(pk.q_o_coeffs, ce * qae);
        push(pk.q_4_coeffs, de * qae);
        push(pk.q_hl_coeffs, p5(ae) * qae);
        push(pk.q_hr_coeffs, p5(be) * qae);
        push(pk.q_h4_coeffs, p5(de) * qae);
        push(pk.q_c_coeffs, qae);
        // custom gates (linearisation_poly.rs:396-430): selector * constraints(evals)
        {
            const CustomEvaluationsC *ce_ = &ev->custom_evals;
            WidgetVals wv;
            wv.a = ae;
            wv.b = be;
            wv.c = ce;
            wv.d = de;
            wv.a_next = ld(ce_->a_next_eval);
            wv.b_next = ld(ce_->b_next_eval);
            wv.d_next = ld(ce_->d_next_eval);
            wv.q_l = ld(ce_->q_l_eval);
            wv.q_r = ld(ce_->q_r_eval);
            wv.q_c = ld(ce_->q_c_eval);
            if (ctx->pk_custom_nz[0]) push(pk.range_selector_coeffs, w_range(range_c, wv));
            if (ctx->pk_custom_nz[1]) push(pk.logic_selector_coeffs, w_logic(logic_c, wv));
            if (ctx->pk_custom_nz[2]) push(pk.fixed_group_add_selector_coeffs, w_fbsm(fixed_c, wv));
            if (ctx->pk_custom_nz[3]) push(pk.variable_group_add_selector_coeffs, w_cadd(var_c, wv));
        }
        // compute_linearisation_permutation (proof_system/permutation.cu:231-265)
        {
            Fr bz = beta * zc;
            Fr a = (ae + bz + gamma) * (be + fr_from_u64(7) * bz + gamma) *
                   (ce + fr_from_u64(13) * bz + gamma) * (de + fr_from_u64(17) * bz + gamma) * alpha;
            push(z_poly, a + l1e * alpha2);
            const Fr s1 = ld(ev->perm_evals.left_sigma_eval), s2 = ld(ev->perm_evals.right_sigma_eval),
                     s3 = ld(ev->perm_evals.out_sigma_eval), pe = ld(ev->perm_evals.permutation_eval);
            Fr b = (ae + beta * s1 + gamma) * (be + beta * s2 + gamma) * (ce + beta * s3 + gamma) *
                   (beta * pe) * alpha;
            push(pk.fourth_sigma_coeffs, neg(b));
        }
        // lookup (widget/lookup.rs:137-182)
        {
            const LookupEvaluationsC *lk = &ev->lookup_evals;
            Fr sep2 = lsep * lsep, sep3 = sep2 * lsep, opd = delta + Fr::one(), eopd = eps * opd;
            if (!ctx->pk_qlookup_zero) {
                Fr ct = ((de * zeta + ce) * zeta + be) * zeta + ae;
                push(pk.q_lookup_coeffs, (ct - ld(lk->f_eval)) * lsep);
            }
            Fr b0 = eps + ld(lk->f_eval);
            Fr b1 = eopd + ld(lk->table_eval) + delta * ld(lk->table_next_eval);
            push(z2_poly, opd * b0 * b1 * sep2 + l1e * sep3);
            if (!h_zero)
                push(h1_poly, neg(ld(lk->z2_next_eval)) * sep2 * (eopd + ld(lk->h2_eval) + delta * ld(lk->h1_next_eval)));
        }
        // - Z_H(z) * sum_k z^(kn) t_(k+1)  (linearisation.cu:250-292)
        {
            Fr p = neg(vh);
            for (int k = 0; k < npieces; k++) {
                push_local(t_poly + 4 * (uint64_t)k * len, p);  // t_poly is range-local
                p = p * zn;
            }
        }
        uint64_t *lin = ctx->buf("lin", len);
        k_lincomb(la, len, lin, s);
        alg((la.k + 1.0) * len);
        if (!dist && nbq < 8) {
            // the verifier's equation (proof.rs:433-494, oracle/verifier.c): for the
            // true quotient lin(z) = -r_0; otherwise the witness does not satisfy
            // the circuit, t has degree >= nbq n and round 4 runs again on all 8
            // blocks (a false pass needs z to be a root of a nonzero polynomial of
            // degree < 8n: probability < 2^-228 over the transcript hash)
            Fr lin_z;
            k_poly_eval(lin, len, zc, ctx->scratch_a, &lin_z, s);
            const LookupEvaluationsC *lk = &ev->lookup_evals;
            Fr pie = Fr::zero();
            const Fr w_inv = inverse(omega);
            for (size_t k = 0; k < pi_pos.size(); k++)
                pie += pi_val[k] * inverse(pow_u64(w_inv, pi_pos[k]) * zc - Fr::one());
            pie = pie * vh * n_inv;
            const Fr *wv[3] = {&ae, &be, &ce};
            const Fr sv[3] = {ld(ev->perm_evals.left_sigma_eval), ld(ev->perm_evals.right_sigma_eval),
                              ld(ev->perm_evals.out_sigma_eval)};
            Fr b = Fr::one();
            for (int j = 0; j < 3; j++) b = b * (*wv[j] + beta * sv[j] + gamma);
            b = b * (de + gamma) * ld(ev->perm_evals.permutation_eval) * alpha;
            const Fr opd = delta + Fr::one(), eopd = eps * opd, sep2 = lsep * lsep, sep3 = sep2 * lsep;
            const Fr h2e = ld(lk->h2_eval);
            const Fr d = sep2 * ld(lk->z2_next_eval) * (eopd + delta * h2e) *
                         (eopd + h2e + delta * ld(lk->h1_next_eval));
            const Fr r0 = pie - b - l1e * alpha2 - d - sep3 * l1e;
            if (!(lin_z + r0).is_zero()) {
                ctx->ktimer.credit("quotient_all_blocks", 1);
                const uint64_t off = 4 * (uint64_t)nbq * n;  // blocks nbq .. 7
                for (int j = 0; j < 4; j++) lde_blocks(nt, wpoly[j], w8buf[j] + off, lg, nbq, 8 - nbq, s, q29);
                lde_blocks(nt, z_poly, z8 + off, lg, nbq, 8 - nbq, s, q29);
                nbq = 8;
                tr = tr3;
                continue;
            }
        }
        tm.mark("r5_lin");

        // transcript appends (gen_proof.cuh:373-403)
        tr.append_scalar("a_eval", ae);
        tr.append_scalar("b_eval", be);
        tr.append_scalar("c_eval", ce);
        tr.append_scalar("d_eval", de);
        tr.append_scalar("left_sig_eval", ld(ev->perm_evals.left_sigma_eval));
        tr.append_scalar("right_sig_eval", ld(ev->perm_evals.right_sigma_eval));
        tr.append_scalar("out_sig_eval", ld(ev->perm_evals.out_sigma_eval));
        tr.append_scalar("perm_eval", ld(ev->perm_evals.permutation_eval));
        const LookupEvaluationsC *lk = &ev->lookup_evals;
        tr.append_scalar("f_eval", ld(lk->f_eval));
        tr.append_scalar("q_lookup_eval", ld(lk->q_lookup_eval));
        tr.append_scalar("lookup_perm_eval", ld(lk->z2_next_eval));
        tr.append_scalar("h_1_eval", ld(lk->h1_eval));
        tr.append_scalar("h_1_next_eval", ld(lk->h1_next_eval));
        tr.append_scalar("h_2_eval", ld(lk->h2_eval));
        const CustomEvaluationsC *cu = &ev->custom_evals;
        tr.append_scalar("q_arith_eval", ld(cu->q_arith_eval));
        tr.append_scalar("q_c_eval", ld(cu->q_c_eval));
        tr.append_scalar("q_l_eval", ld(cu->q_l_eval));
        tr.append_scalar("q_r_eval", ld(cu->q_r_eval));
        tr.append_scalar("q_hl_eval", ld(cu->q_hl_eval));
        tr.append_scalar("q_hr_eval", ld(cu->q_hr_eval));
        tr.append_scalar("q_h4_eval", ld(cu->q_h4_eval));
        tr.append_scalar("a_next_eval", ld(cu->a_next_eval));
        tr.append_scalar("b_next_eval", ld(cu->b_next_eval));
        tr.append_scalar("d_next_eval", ld(cu->d_next_eval));

        // ---------------- round 6: openings (gen_proof.cuh:405-463, kzg10.cu:116-145)
        // Both "aggregate_witness" challenges are squeezed back to back in the
        // reference (nothing is appended in between), so both witness
        // polynomials are built first and committed in one batched MSM.
        uint64_t *comb = ctx->buf("comb", len), *comb2 = ctx->buf("comb2", len);
        Fr aw = tr.challenge_scalar("aggregate_witness");
        Fr saw = tr.challenge_scalar("aggregate_witness");
        {
            const uint64_t *awp[11] = {lin, pk.left_sigma_coeffs, pk.right_sigma_coeffs,
                                       pk.out_sigma_coeffs, f_poly, h2_poly, table_poly,
                                       wpoly[0], wpoly[1], wpoly[2], wpoly[3]};
            LinArgs oa;
            oa.k = 0;
            Fr p = Fr::one();
            for (int k = 0; k < 11; k++) {
                bool skip = (k == 4 && f_zero) || (k == 5 && h_zero) || (k == 6 && table_zero);
                if (!skip) {
                    oa.p[oa.k] = k == 0 ? awp[k] : awp[k] + 4 * q0;  // lin is range-local
                    oa.s[oa.k] = p;
                    oa.k++;
                }
                p = p * aw;
            }
            k_lincomb(oa, len, comb, s);
            alg((oa.k + 1.0) * len);
        }
        {
            const uint64_t *sawp[7] = {z_poly, wpoly[0], wpoly[1], wpoly[3], h1_poly, z2_poly, table_poly};
            LinArgs oa;
            oa.k = 0;
            Fr p = Fr::one();
            for (int k = 0; k < 7; k++) {
                bool skip = (k == 4 && h_zero) || (k == 6 && table_zero);
                if (!skip) {
                    oa.p[oa.k] = sawp[k] + 4 * q0;
                    oa.s[oa.k] = p;
                    oa.k++;
                }
                p = p * saw;
            }
            k_lincomb(oa, len, comb2, s);
            alg((oa.k + 1.0) * len + 4.0 * len);  // + both divisions
        }
        {
            uint64_t *dd[2] = {comb, comb2};
            const Fr zz[2] = {zc, zw};
            div_linear_range(ctx, dd, zz, 2, len, dist);
        }
        tm.mark("r6_witness");
        {
            const uint64_t *sc[2] = {comb, comb2};
            CommitmentC *oc[2] = {&out->aw_opening, &out->saw_opening};
            commit_affine_batch(ctx, sc, 2, n, oc, dist);
        }
        tm.mark("r6_commit");
        break;
    }
    // the tables this proof went without: built in the background from now
    if (bg_mode && ctx->defer_now && ctx->tables_wanted) tables_start_background(ctx, n);
    return PNP_OK;
}

}  // namespace pnp
