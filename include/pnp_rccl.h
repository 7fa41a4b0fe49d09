/* pnp_rccl.h — native RCCL exchange for multi-GPU gen_proof (libpnp_rccl.so).
 *
 * The multi-GPU prover (include/pnp_plonk.h, "Multi-GPU") reaches its three
 * collectives through callbacks: the point-range / control all-gathers
 * (pnp_set_msm_shard), the round-4 all-to-all (pnp_set_exchange_a2a) and the
 * bucket-range variable all-to-all (pnp_set_exchange_v).  This library
 * implements them on RCCL over xGMI, enqueued on the prover's own stream
 * (pnp_ctx_stream) with no host synchronisation (pnp_set_exchange_ordered), so
 * a host without Python — the reference's Rust Prover::prove_pnp
 * (plonk-core/src/proof_system/prover.rs:902) — gets the north star's RCCL path
 * with a 128-byte id to hand around and one call per rank:
 *
 *     rank 0:        pnp_rccl_unique_id(id);  ... send id to every rank ...
 *     every rank r:  hipSetDevice(local); pnp_ctx_create(local, &ctx);
 *                    pnp_rccl_attach(ctx, r, world, id, 0, 0, 0, &ex);
 *                    pnp_load_prover_key(...); pnp_load_commit_key(...);
 *                    pnp_prove(...)  ... pnp_rccl_detach(ex); pnp_ctx_destroy(ctx);
 *
 * It is a separate shared object so that a process that already maps an RCCL
 * (torch's bundled one) never loads a second: torch hosts keep pnp/shard.py.
 * The reference proves on one GPU; there is no reference counterpart. */
#ifndef PNP_RCCL_H
#define PNP_RCCL_H
#include <stdint.h>
#include "pnp_plonk.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pnp_rccl pnp_rccl;

#define PNP_RCCL_ID_BYTES 128

/* A new communicator id (ncclGetUniqueId), made by one rank and handed to all. */
int pnp_rccl_unique_id(uint8_t id[PNP_RCCL_ID_BYTES]);

/* Joins the communicator (ncclCommInitRank on the context's device),
 * allocates the exchange buffers on that device and registers the callbacks
 * with ctx: pnp_set_msm_shard (all-gather slots of xbuf_bytes), and when
 * world divides 8 pnp_set_exchange_a2a (a2a_bytes), and when v_bytes > 0
 * pnp_set_exchange_v (bucket-range records, v_bytes each way); 0 picks the
 * sizes pnp/shard.py uses for the context's later key (n = 2^lg_hint when
 * lg_hint > 0, else 2^22).  Call before pnp_load_prover_key.  world = 1: a
 * communicator of one (every collective an identity; the prover does not
 * call them). */
int pnp_rccl_attach(pnp_ctx *ctx, int rank, int world, const uint8_t id[PNP_RCCL_ID_BYTES], uint32_t lg_hint,
                    uint64_t a2a_bytes, uint64_t v_bytes, pnp_rccl **out);

/* Unregisters the exchanges from the context (back to one GPU), frees the
 * buffers and destroys the communicator. */
int pnp_rccl_detach(pnp_rccl *ex);

/* The callbacks themselves, callable directly (tests): they enqueue on the
 * context's stream and return; pnp_rccl_buffers reports the device buffers
 * (xbuf, a2a, vsend, vrecv) and their sizes. */
int pnp_rccl_allgather(void *ex, uint64_t bytes_per_rank);
int pnp_rccl_alltoall(void *ex, uint64_t bytes_per_peer);
int pnp_rccl_alltoallv(void *ex, const uint64_t *send_bytes, const uint64_t *recv_bytes);
int pnp_rccl_buffers(pnp_rccl *ex, void *bufs[4], uint64_t bytes[4]);
/* calls made so far: all-gathers, all-to-alls, variable all-to-alls */
int pnp_rccl_calls(pnp_rccl *ex, uint64_t calls[3]);

#ifdef __cplusplus
}
#endif
#endif
