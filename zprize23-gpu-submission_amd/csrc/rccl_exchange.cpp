// rccl_exchange.cpp — libpnp_rccl.so: the multi-GPU prover's exchanges on
// RCCL, enqueued on the prover's stream (include/pnp_rccl.h).
//
// The prover calls three collectives through callbacks (include/pnp_plonk.h,
// "Multi-GPU"); each is one RCCL call here, on the context's stream, so the
// data it moves is ordered behind the kernels that produced it and the
// library's next copies / kernels behind the collective — no host
// synchronisation and no Python in between (pnp/shard.py, the torch host's
// exchange, synchronises after every collective):
//   * all-gather of the per-rank slots (point-range MSM partial sums, the
//     tagged control words): in-place ncclAllGather on xbuf;
//   * round-4 all-to-all (blocks -> coefficient ranges): ncclAllToAll from the
//     send slots to the receive slots of the a2a buffer;
//   * bucket-range records: ncclAllToAllv with the library's byte counts.
// xGMI is point-to-point (7 links per GPU): RCCL's all-to-all sends every
// peer's segment on its own link, the all-gather is a ring over the slots.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <string.h>
#include <new>
#include <vector>
#include "../../include/pnp_rccl.h"

struct pnp_rccl {
    pnp_ctx *ctx = nullptr;
    ncclComm_t comm = nullptr;
    hipStream_t s = nullptr;
    int rank = 0, world = 1;
    void *buf[4] = {nullptr, nullptr, nullptr, nullptr};  // xbuf, a2a, vsend, vrecv
    uint64_t bytes[4] = {0, 0, 0, 0};
    uint64_t calls[3] = {0, 0, 0};
};

namespace {

constexpr uint64_t XBUF_BYTES = 1 << 20;  // all-gather slots (as pnp/shard.py)

int fail(const char *what, ncclResult_t r) {
    fprintf(stderr, "pnp_rccl: %s: %s\n", what, ncclGetErrorString(r));
    return PNP_E_DEVICE;
}

// pnp/shard.py a2a_bytes_for / v_bytes_for
uint64_t a2a_bytes_for(uint32_t lg, int world) {
    if (world <= 1 || 8 % world) return 0;
    const uint64_t n = 1ULL << lg;
    return 2ULL * world * (8 / world) * (n / world) * 32;
}
uint64_t v_bytes_for(uint32_t lg, int world) {
    if (world <= 1) return 0;
    const int c = lg >= 19 ? 20 : (lg > 7 ? (int)lg - 3 : 4);
    const uint64_t windows = (256 + c - 1) / c, per = ((1ULL << lg) + world - 1) / world;
    return 2 * 8 * windows * per * 8;
}

}  // namespace

extern "C" {

int pnp_rccl_unique_id(uint8_t id[PNP_RCCL_ID_BYTES]) {
    if (!id) return PNP_E_ARG;
    ncclUniqueId u;
    static_assert(sizeof u == PNP_RCCL_ID_BYTES, "ncclUniqueId is 128 bytes");
    if (ncclResult_t r = ncclGetUniqueId(&u)) return fail("ncclGetUniqueId", r);
    memcpy(id, &u, sizeof u);
    return PNP_OK;
}

int pnp_rccl_allgather(void *u, uint64_t b) {
    auto *e = static_cast<pnp_rccl *>(u);
    if (!e || b * e->world > e->bytes[0]) return PNP_E_ARG;
    char *x = static_cast<char *>(e->buf[0]);
    // in place: rank r's slot is its send buffer
    if (ncclResult_t r = ncclAllGather(x + e->rank * b, x, b, ncclUint8, e->comm, e->s))
        return fail("ncclAllGather", r);
    e->calls[0]++;
    return PNP_OK;
}

int pnp_rccl_alltoall(void *u, uint64_t b) {
    auto *e = static_cast<pnp_rccl *>(u);
    if (!e || 2 * b * e->world > e->bytes[1]) return PNP_E_ARG;
    char *a = static_cast<char *>(e->buf[1]);
    if (ncclResult_t r = ncclAllToAll(a, a + b * e->world, b, ncclUint8, e->comm, e->s))
        return fail("ncclAllToAll", r);
    e->calls[1]++;
    return PNP_OK;
}

int pnp_rccl_alltoallv(void *u, const uint64_t *send_bytes, const uint64_t *recv_bytes) {
    auto *e = static_cast<pnp_rccl *>(u);
    if (!e || !send_bytes || !recv_bytes) return PNP_E_ARG;
    const int W = e->world;
    std::vector<size_t> sc(W), sd(W), rc(W), rd(W);
    uint64_t so = 0, ro = 0;
    for (int j = 0; j < W; j++) {  // 8-byte records: counts in u64 elements
        if (send_bytes[j] % 8 || recv_bytes[j] % 8) return PNP_E_ARG;
        sc[j] = send_bytes[j] / 8, sd[j] = so, so += sc[j];
        rc[j] = recv_bytes[j] / 8, rd[j] = ro, ro += rc[j];
    }
    if (8 * so > e->bytes[2] || 8 * ro > e->bytes[3]) return PNP_E_ARG;
    if (ncclResult_t r = ncclAllToAllv(e->buf[2], sc.data(), sd.data(), e->buf[3], rc.data(), rd.data(), ncclUint64,
                                       e->comm, e->s))
        return fail("ncclAllToAllv", r);
    e->calls[2]++;
    return PNP_OK;
}

int pnp_rccl_attach(pnp_ctx *ctx, int rank, int world, const uint8_t id[PNP_RCCL_ID_BYTES], uint32_t lg_hint,
                    uint64_t a2a_bytes, uint64_t v_bytes, pnp_rccl **out) {
    if (!ctx || !id || !out || world < 1 || rank < 0 || rank >= world) return PNP_E_ARG;
    *out = nullptr;
    pnp_rccl *e = new (std::nothrow) pnp_rccl;
    if (!e) return PNP_E_NOMEM;
    e->ctx = ctx, e->rank = rank, e->world = world;
    void *sp = nullptr;
    int rc = pnp_ctx_stream(ctx, &sp);
    if (rc) {
        delete e;
        return rc;
    }
    e->s = static_cast<hipStream_t>(sp);
    int dev = 0;
    if (hipStreamGetDevice(e->s, &dev) != hipSuccess || hipSetDevice(dev) != hipSuccess) {
        delete e;
        return PNP_E_DEVICE;
    }
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    if (ncclResult_t r = ncclCommInitRank(&e->comm, world, u, rank)) {
        delete e;
        return fail("ncclCommInitRank", r);
    }
    const uint32_t lg = lg_hint ? lg_hint : 22;
    e->bytes[0] = XBUF_BYTES;
    e->bytes[1] = a2a_bytes ? a2a_bytes : a2a_bytes_for(lg, world);
    // bucket ranges pay from 4 ranks on (msm.hip msm_bucket_batch); below
    // that the folded tables stay per point range
    e->bytes[2] = e->bytes[3] = v_bytes ? v_bytes : (world >= 4 ? v_bytes_for(lg, world) : 0);
    for (int k = 0; k < 4; k++) {
        if (!e->bytes[k]) continue;
        if (hipMalloc(&e->buf[k], e->bytes[k]) != hipSuccess || hipMemset(e->buf[k], 0, e->bytes[k]) != hipSuccess) {
            (void)hipGetLastError();
            pnp_rccl_detach(e);
            return PNP_E_NOMEM;
        }
    }
    if (world > 1) {
        rc = pnp_set_msm_shard(ctx, rank, world, pnp_rccl_allgather, e, static_cast<uint64_t *>(e->buf[0]),
                               e->bytes[0]);
        if (!rc && e->bytes[1])
            rc = pnp_set_exchange_a2a(ctx, pnp_rccl_alltoall, e, static_cast<uint64_t *>(e->buf[1]), e->bytes[1]);
        if (!rc && e->bytes[2])
            rc = pnp_set_exchange_v(ctx, pnp_rccl_alltoallv, e, static_cast<uint64_t *>(e->buf[2]),
                                    static_cast<uint64_t *>(e->buf[3]), e->bytes[2]);
        if (!rc) rc = pnp_set_exchange_ordered(ctx, 1);
        if (rc) {
            pnp_rccl_detach(e);
            return rc;
        }
    }
    *out = e;
    return PNP_OK;
}

int pnp_rccl_detach(pnp_rccl *e) {
    if (!e) return PNP_E_ARG;
    if (e->ctx && e->world > 1) {
        pnp_set_exchange_ordered(e->ctx, 0);
        pnp_set_exchange_v(e->ctx, nullptr, nullptr, nullptr, nullptr, 0);
        pnp_set_exchange_a2a(e->ctx, nullptr, nullptr, nullptr, 0);
        pnp_set_msm_shard(e->ctx, 0, 1, nullptr, nullptr, nullptr, 0);
    }
    if (e->s) (void)hipStreamSynchronize(e->s);
    for (void *&b : e->buf) {
        if (b) (void)hipFree(b);
        b = nullptr;
    }
    if (e->comm) ncclCommDestroy(e->comm);
    delete e;
    return PNP_OK;
}

int pnp_rccl_buffers(pnp_rccl *e, void *bufs[4], uint64_t bytes[4]) {
    if (!e || !bufs || !bytes) return PNP_E_ARG;
    for (int k = 0; k < 4; k++) bufs[k] = e->buf[k], bytes[k] = e->bytes[k];
    return PNP_OK;
}

int pnp_rccl_calls(pnp_rccl *e, uint64_t calls[3]) {
    if (!e || !calls) return PNP_E_ARG;
    for (int k = 0; k < 3; k++) calls[k] = e->calls[k];
    return PNP_OK;
}

}  // extern "C"
