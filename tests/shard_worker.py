"""One rank of the multi-process sharding tests (tests/test_shard.py).

    RANK=r WORLD_SIZE=N MASTER_ADDR=127.0.0.1 MASTER_PORT=p \
        python shard_worker.py {cpu|gpu} OUT_PREFIX [lg seed]
        python shard_worker.py full OUT_PREFIX lg gates seed
        python shard_worker.py hbm OUT_PREFIX lg seed   (PNP_TEST_SHORT_RANK)

cpu: exercises pnp.shard.WindowExchange over gloo with host tensors.
gpu: every rank proves the same seeded instance on cuda:0 with point-range
     sharded MSMs and, when world divides 8, the distributed round 4 (gloo
     exchanges through host memory, since the ranks share one GPU) and writes
     its ProofC bytes to OUT_PREFIX.<rank>.
full: the same over bench.Synthetic at full size (keys GPU-resident)."""
import ctypes as C
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "zprize23-gpu-submission_amd"))


def _v_bytes(lg, world):
    """PNP_TEST_MSM_SHARD=points: point-range MSMs; default: bucket ranges"""
    from pnp.shard import v_bytes_for
    return 0 if os.environ.get("PNP_TEST_MSM_SHARD") == "points" else v_bytes_for(lg, world)


def main():
    mode, out = sys.argv[1], sys.argv[2]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pnp.shard import WindowExchange
    if mode == "cpu":
        ex = WindowExchange(rank, world, capacity_bytes=1 << 14)
        for w in (24, 24 * 7, 8):  # slot sizes in u64 words (window sums are 24 words)
            ex.buf.zero_()
            ex.buf[rank * w:(rank + 1) * w] = torch.arange(w) + 1000 * (rank + 1)
            ex.gather(w * 8)
            exp = torch.cat([torch.arange(w) + 1000 * (r + 1) for r in range(world)])
            assert torch.equal(ex.buf[:w * world], exp), (w, ex.buf[:w * world])
            assert int(ex.buf[w * world:].abs().sum()) == 0
        # all-to-all: slot s of rank r carries (r, s); afterwards receive slot s
        # holds what rank s sent to this rank
        ex2 = WindowExchange(rank, world, capacity_bytes=1 << 12, a2a_bytes=2 * world * 5 * 8)
        for s in range(world):
            ex2.a2a[5 * s:5 * s + 5] = torch.arange(5) + 100 * rank + 10 * s
        ex2.alltoall(5 * 8)
        for s in range(world):
            got = ex2.a2a[5 * (world + s):5 * (world + s) + 5]
            assert torch.equal(got, torch.arange(5) + 100 * s + 10 * rank), (s, got)
        # variable all-to-all (bucket-range MSMs): rank r sends (r + 1) * (s + 1)
        # words to rank s, valued 1000 r + s
        ex3 = WindowExchange(rank, world, capacity_bytes=1 << 12, v_bytes=1 << 12)
        send = [(rank + 1) * (s + 1) for s in range(world)]
        at = 0
        for s_, k in enumerate(send):
            ex3.vsend[at:at + k] = 1000 * rank + s_
            at += k
        recv = [(r + 1) * (rank + 1) for r in range(world)]
        ex3.alltoallv([8 * k for k in send], [8 * k for k in recv])
        at = 0
        for r, k in enumerate(recv):
            assert torch.equal(ex3.vrecv[at:at + k], torch.full((k,), 1000 * r + rank)), (r, ex3.vrecv[at:at + k])
            at += k
        cbv = ex3.c_alltoallv()
        arr = C.c_uint64 * world
        assert cbv(None, arr(*[8 * k for k in send]), arr(*[8 * k for k in recv])) == 0 and ex3.v_calls == 2
        cb = ex.c_callback()
        assert cb(None, 24 * 8) == 0 and ex.calls == 4
        assert cb(None, 1 << 20) == 1 and ex.error is not None  # oversize slot -> error code
        with open(f"{out}.{rank}", "w") as f:
            f.write("ok")
    elif mode == "hbm":
        # one rank short of HBM (PNP_TEST_SHORT_RANK): every rank's first
        # proof must fail with PNP_E_NOMEM naming that rank, before any work
        # (abi.cpp hbm_budget)
        short = int(os.environ["PNP_TEST_SHORT_RANK"])
        if rank == short:
            os.environ["PNP_HBM_LIMIT"] = "1"
        lg, seed = int(sys.argv[3]), int(sys.argv[4])
        import pnp
        from pnp_testlib import Inputs
        from pnp.shard import a2a_bytes_for
        inp = Inputs(lg, seed)
        ctx = pnp.Context(0)
        ex = WindowExchange(rank, world, device="cuda", a2a_bytes=a2a_bytes_for(lg, world),
                            v_bytes=_v_bytes(lg, world))
        ctx.set_msm_shard(ex)
        ctx.load_prover_key(inp.pk, inp.n, device_ptrs=False)
        ctx.load_commit_key(inp.ck, inp.n, device_ptrs=False)
        try:
            ctx.prove(inp.circuit, device_ptrs=False)
            msg = "proved"
        except pnp.PnpError as e:
            msg = str(e)
        assert "PNP_E_NOMEM" in msg and f"rank {short} of {world}" in msg, msg
        with open(f"{out}.{rank}", "w") as f:
            f.write("ok")
        ctx.close()
    elif mode == "full":
        # bench.Synthetic (the HEIGHT=15 instance, GPU-generated) at full size
        lg, gates, seed = int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
        circuit = sys.argv[6] if len(sys.argv) > 6 else "arith"
        sys.path.insert(0, os.path.dirname(HERE))
        import pnp
        from pnp import abi
        from bench import Synthetic
        from pnp.shard import a2a_bytes_for
        import time
        t0 = time.time()
        def say(what):
            f_, t_ = torch.cuda.mem_get_info()
            print(f"rank {rank}: {what} ({time.time() - t0:.1f} s, HBM free {f_ / 2**30:.1f} GiB)", flush=True)
        ctx = pnp.Context(0)
        ex = WindowExchange(rank, world, device="cuda", a2a_bytes=a2a_bytes_for(lg, world),
                            v_bytes=_v_bytes(lg, world))
        ctx.set_msm_shard(ex)
        say("context")
        syn = Synthetic(ctx, lg, gates, seed=seed, circuit=circuit)
        say("instance")
        ctx.load_prover_key(syn.pk, syn.n, device_ptrs=True)
        ctx.load_commit_key(syn.ck, syn.n, device_ptrs=True)
        plan = ctx.hbm_usage()
        say(f"keys loaded, hbm {plan}")
        # the context keeps block-layout copies of this rank's 8n evaluations
        # and never reads the caller's 8n arrays again: free them, so that 8
        # ranks fit one GPU's HBM
        for k in [k for k, t in syn.keep.items() if t.shape[0] == 8 * syn.n]:
            del syn.keep[k]
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        groups = os.environ.get("PNP_EXPECT_GROUPS") == "1"
        report = os.environ.get("PNP_REPORT_GROUPS") == "1"  # record, do not assert (the test decides)
        if groups or report:
            ctx.kernel_timing(True)
        say("proving")
        try:
            proof = ctx.prove(syn.cs, device_ptrs=True)
        except Exception:
            print(f"rank {rank}: exchange error: {ex.error!r}", flush=True)
            raise
        say(f"proved, hbm {ctx.hbm_usage()}")
        if groups:  # the wires and z were committed over their groups
            assert ctx.kernel_bytes("wire_groups_used") == 1, ctx.kernel_bytes("wire_groups_used")
            assert ctx.kernel_bytes("z_groups_used") == 1, ctx.kernel_bytes("z_groups_used")
            ctx.kernel_timing(False)
        elif report:
            import json
            f_, t_ = torch.cuda.mem_get_info()
            with open(f"{out}.{rank}.groups", "w") as fh:
                json.dump({"wire_groups_used": ctx.kernel_bytes("wire_groups_used"),
                           "z_groups_used": ctx.kernel_bytes("z_groups_used"), "plan": plan,
                           "hbm_total": t_}, fh)
            ctx.kernel_timing(False)
        assert ex.calls > 0
        assert (ex.a2a_calls > 0) == (8 % world == 0)
        if os.environ.get("PNP_EXPECT_BUCKETS"):
            assert (ex.v_calls > 0) == (os.environ["PNP_EXPECT_BUCKETS"] == "1"), ex.v_calls
        again = _prove_again(ctx, ex, lambda: ctx.prove(syn.cs, device_ptrs=True), proof)
        say(f"second proof: {again}")
        with open(f"{out}.{rank}", "wb") as f:
            f.write(abi.proof_to_bytes(proof))
        ctx.close()
    else:
        lg, seed = int(sys.argv[3]), int(sys.argv[4])
        import pnp
        from pnp import abi
        from pnp_testlib import Inputs
        inp = Inputs(lg, seed)
        ctx = pnp.Context(0)
        from pnp.shard import a2a_bytes_for
        ex = WindowExchange(rank, world, device="cuda", a2a_bytes=a2a_bytes_for(lg, world),
                            v_bytes=_v_bytes(lg, world))
        ctx.set_msm_shard(ex)
        ctx.load_prover_key(inp.pk, inp.n, device_ptrs=False)
        ctx.load_commit_key(inp.ck, inp.n, device_ptrs=False)
        proof = ctx.prove(inp.circuit, device_ptrs=False)
        assert ex.calls > 0
        assert (ex.a2a_calls > 0) == (8 % world == 0)
        # bucket ranges whenever the bucket count splits (not 3 ranks, not tiny MSMs)
        if os.environ.get("PNP_EXPECT_BUCKETS"):
            assert (ex.v_calls > 0) == (os.environ["PNP_EXPECT_BUCKETS"] == "1"), ex.v_calls
        _prove_again(ctx, ex, lambda: ctx.prove(inp.circuit, device_ptrs=False), proof)
        with open(f"{out}.{rank}", "wb") as f:
            f.write(abi.proof_to_bytes(proof))
        ctx.close()
    dist.destroy_process_group()


def _prove_again(ctx, ex, prove, first):
    """A second proof on the same context must give the same bytes.  In
    bucket-range mode it moves its records through the fixed-slot exchange
    (capacities learned from the first proof, msm.hip msm_bucket_batch): every
    batch slotted, none redone — unless PNP_TEST_SLOT_CAP shrinks the slots,
    when every batch overflows, is redone on the variable path and the bytes
    still match."""
    from pnp import abi
    ctx.kernel_timing(True)
    proof = prove()
    slotted, over = ctx.kernel_bytes("msm_slot_batches"), ctx.kernel_bytes("msm_slot_overflows")
    ctx.kernel_timing(False)
    assert abi.proof_to_bytes(proof) == abi.proof_to_bytes(first), "second proof differs"
    if os.environ.get("PNP_EXPECT_BUCKETS") == "1":
        if os.environ.get("PNP_TEST_SLOT_CAP"):
            assert over > 0 and slotted == 0, (slotted, over)
        else:
            assert slotted > 0 and over == 0, (slotted, over)
    return {"slotted": slotted, "overflows": over, "v_calls": ex.v_calls}


if __name__ == "__main__":
    main()
