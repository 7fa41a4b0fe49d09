"""libpnp_rccl.so at world size 1, in a process that never imports torch (the
way a Rust host would run it): ctypes over the two libraries and the HIP
runtime only.  Run by tests/test_gpu_rccl.py::test_native_rccl_world1.

The same assertions as the torch exchange test (test_rccl_exchange_world1):
every collective of a one-rank communicator is an identity — the in-place
all-gather of the slots, the even all-to-all (send slots -> receive slots),
the variable all-to-all with split sizes — here enqueued on the prover's own
stream with no host synchronisation inside the callbacks; then a proof on the
context with the exchange attached equals the CPU restatement's."""
import ctypes as C
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "zprize23-gpu-submission_amd"))

import numpy as np  # noqa: E402

from pnp import abi  # noqa: E402  (ctypes structs only: no torch)

LIB = os.path.join(os.path.dirname(HERE), "zprize23-gpu-submission_amd", "lib")


def main():
    assert "torch" not in sys.modules
    plonk = C.CDLL(os.path.join(LIB, "libpnp_plonk.so"), mode=C.RTLD_GLOBAL)
    rccl = C.CDLL(os.path.join(LIB, "libpnp_rccl.so"))
    hip = C.CDLL("libamdhip64.so.7")
    vp, u64 = C.c_void_p, C.c_uint64
    hip.hipMemcpy.argtypes = [vp, vp, C.c_size_t, C.c_int]
    H2D, D2H = 1, 2
    plonk.pnp_ctx_create.argtypes = [C.c_int, C.POINTER(vp)]
    plonk.pnp_sync.argtypes = [vp]
    plonk.pnp_last_error.restype = C.c_char_p
    rccl.pnp_rccl_attach.argtypes = [vp, C.c_int, C.c_int, C.c_char_p, C.c_uint32, u64, u64, C.POINTER(vp)]
    rccl.pnp_rccl_buffers.argtypes = [vp, C.POINTER(vp), C.POINTER(u64)]
    rccl.pnp_rccl_calls.argtypes = [vp, C.POINTER(u64)]
    rccl.pnp_rccl_allgather.argtypes = [vp, u64]
    rccl.pnp_rccl_alltoall.argtypes = [vp, u64]
    rccl.pnp_rccl_alltoallv.argtypes = [vp, C.POINTER(u64), C.POINTER(u64)]
    rccl.pnp_rccl_detach.argtypes = [vp]

    ctx = vp()
    assert plonk.pnp_ctx_create(0, C.byref(ctx)) == 0
    uid = C.create_string_buffer(128)
    assert rccl.pnp_rccl_unique_id(uid) == 0
    ex = vp()
    rc = rccl.pnp_rccl_attach(ctx, 0, 1, uid.raw, 10, 2 * 4096 * 8, 10000 * 8, C.byref(ex))
    assert rc == 0, rc
    bufs, sizes = (vp * 4)(), (u64 * 4)()
    assert rccl.pnp_rccl_buffers(ex, bufs, sizes) == 0
    assert list(sizes) == [1 << 20, 2 * 4096 * 8, 10000 * 8, 10000 * 8], list(sizes)

    def put(dev, arr):
        assert hip.hipMemcpy(dev, arr.ctypes.data, arr.nbytes, H2D) == 0

    def get(dev, count):
        out = np.zeros(count, dtype=np.int64)
        assert plonk.pnp_sync(ctx) == 0  # the collectives ran on the prover's stream
        assert hip.hipMemcpy(out.ctypes.data, dev, out.nbytes, D2H) == 0
        return out

    rng = np.random.default_rng(5)
    # all-gather slots: B x 192 B partial sums
    x = (np.arange(48, dtype=np.int64) * 7 + 1)
    put(bufs[0], x)
    assert rccl.pnp_rccl_allgather(ex, 48 * 8) == 0
    assert (get(bufs[0], 48) == x).all()
    # even all-to-all: send slots then receive slots
    a = rng.integers(-2**62, 2**62, 4096, dtype=np.int64)
    put(bufs[1], a)
    assert rccl.pnp_rccl_alltoall(ex, 4096 * 8) == 0
    assert (get(C.c_void_p(bufs[1] + 4096 * 8), 4096) == a).all()
    # variable all-to-all with split sizes (bucket-range records)
    v = rng.integers(-2**62, 2**62, 10000, dtype=np.int64)
    put(bufs[2], v)
    put(bufs[3], np.zeros(10000, dtype=np.int64))
    cnt = (u64 * 1)(7777 * 8)
    assert rccl.pnp_rccl_alltoallv(ex, cnt, cnt) == 0
    got = get(bufs[3], 10000)
    assert (got[:7777] == v[:7777]).all() and not got[7777:].any()
    # oversize requests are refused, nothing enqueued
    assert rccl.pnp_rccl_allgather(ex, 1 << 21) != 0
    calls = (u64 * 3)()
    assert rccl.pnp_rccl_calls(ex, calls) == 0 and list(calls) == [1, 1, 1], list(calls)

    # a proof on the context with the exchange attached (world 1: the prover
    # never calls it) equals the CPU restatement's
    from pnp_testlib import Inputs
    inp = Inputs(8, 11)
    exp = abi.proof_to_bytes(inp.oracle_proof())
    plonk.pnp_load_prover_key.argtypes = [vp, C.POINTER(abi.ProverKeyC), u64, C.c_int]
    plonk.pnp_load_commit_key.argtypes = [vp, C.POINTER(abi.CommitKeyC), u64, C.c_int]
    plonk.pnp_prove.argtypes = [vp, C.POINTER(abi.CircuitC), C.c_int, C.POINTER(abi.ProofC)]
    assert plonk.pnp_load_prover_key(ctx, C.byref(inp.pk), inp.n, 0) == 0, plonk.pnp_last_error()
    assert plonk.pnp_load_commit_key(ctx, C.byref(inp.ck), inp.n, 0) == 0, plonk.pnp_last_error()
    out = abi.ProofC()
    assert plonk.pnp_prove(ctx, C.byref(inp.circuit), 0, C.byref(out)) == 0, plonk.pnp_last_error()
    assert abi.proof_to_bytes(out) == exp
    assert rccl.pnp_rccl_detach(ex) == 0
    plonk.pnp_ctx_destroy.argtypes = [vp]
    plonk.pnp_ctx_destroy(ctx)
    assert "torch" not in sys.modules
    print("native rccl world-1 exchange ok")


if __name__ == "__main__":
    main()
