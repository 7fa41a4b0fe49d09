"""RCCL (torch.distributed backend "nccl") on the exchange paths of
pnp/shard.py, at world size 1.

The pool gives one GPU per box and RCCL refuses two ranks on one device, so
the multi-rank proofs are rehearsed with gloo (tests/test_shard.py).  This
test runs the very calls the 8-GPU bench makes on device buffers —
`all_gather_into_tensor` (MSM partial sums, scalar slots),
`all_to_all_single` even (round-4 blocks) and with split sizes (bucket-range
records), and the bench's float64 `all_reduce(MAX)` — through a real RCCL
communicator, so dtype, contiguity and stream handling are checked on the
library that the driver's multi-GPU run loads.  With one rank every
collective is an identity, which is what the test asserts."""
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(HERE), "zprize23-gpu-submission_amd")

WORKER = r"""
import sys, torch, torch.distributed as dist
sys.path.insert(0, sys.argv[1])
from pnp.shard import WindowExchange
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=dev)
ex = WindowExchange(0, 1, device=dev)
ex.backend = dist.get_backend()          # world 1: the constructor leaves it "none"
assert ex.backend == "nccl", ex.backend
# all-gather slots: B x 192 B partial sums
ex.buf[:48].copy_(torch.arange(48, dtype=torch.int64, device=dev) * 7 + 1)
ex.gather(48 * 8)
assert torch.equal(ex.buf[:48].cpu(), torch.arange(48, dtype=torch.int64) * 7 + 1)
# even all-to-all: send slots then receive slots
ex.a2a = torch.zeros(2 * 4096, dtype=torch.int64, device=dev)
ex.a2a[:4096].copy_(torch.randint(-2**62, 2**62, (4096,), dtype=torch.int64))
ex.alltoall(4096 * 8)
assert torch.equal(ex.a2a[4096:], ex.a2a[:4096])
# variable all-to-all with split sizes (bucket-range records)
ex.vsend = torch.randint(-2**62, 2**62, (10000,), dtype=torch.int64, device=dev)
ex.vrecv = torch.zeros(10000, dtype=torch.int64, device=dev)
ex.alltoallv([7777 * 8], [7777 * 8])
assert torch.equal(ex.vrecv[:7777], ex.vsend[:7777]) and int(ex.vrecv[7777:].abs().sum()) == 0
# the ctypes trampolines the library calls
cb, cba, cbv = ex.c_callback(), ex.c_alltoall(), ex.c_alltoallv()
assert cb(None, 48 * 8) == 0 and cba(None, 4096 * 8) == 0
import ctypes
arr = (ctypes.c_uint64 * 1)(7777 * 8)
assert cbv(None, arr, arr) == 0 and ex.error is None
assert (ex.calls, ex.a2a_calls, ex.v_calls) == (2, 2, 2)
# stream-ordered: the collectives enqueued on another stream (the library's,
# pnp.Context.set_msm_shard), no host synchronisation; the results appear once
# that stream is synchronised
side = torch.cuda.Stream()
ex.stream = torch.cuda.ExternalStream(side.cuda_stream)
assert ex.ordered
with torch.cuda.stream(side):
    ex.buf[:24].copy_(torch.arange(24, dtype=torch.int64, device=dev) - 5)
    ex.a2a[:4096].copy_(torch.arange(4096, dtype=torch.int64, device=dev) * 3)
ex.gather(24 * 8)
ex.alltoall(4096 * 8)
ex.alltoallv([1000 * 8], [1000 * 8])
side.synchronize()
assert torch.equal(ex.buf[:24].cpu(), torch.arange(24, dtype=torch.int64) - 5)
assert torch.equal(ex.a2a[4096:].cpu(), torch.arange(4096, dtype=torch.int64) * 3)
assert torch.equal(ex.vrecv[:1000], ex.vsend[:1000])
assert (ex.calls, ex.a2a_calls, ex.v_calls) == (3, 3, 3)
# the bench's max-over-ranks timing
t = torch.tensor([1.25], dtype=torch.float64, device=dev)
dist.all_reduce(t, op=dist.ReduceOp.MAX)
assert float(t.item()) == 1.25
dist.destroy_process_group()
print("rccl world-1 exchange ok")
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_rccl_exchange_world1(tmp_path):
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    log = tmp_path / "rccl.log"
    with open(log, "wb") as f:
        p = subprocess.run([sys.executable, "-c", WORKER, PKG], env=env, stdout=f,
                           stderr=subprocess.STDOUT, timeout=110)
    out = log.read_text(errors="replace")
    assert p.returncode == 0, out[-3000:]
    assert "rccl world-1 exchange ok" in out


@pytest.mark.gpu
def test_native_rccl_world1(tmp_path):
    """libpnp_rccl.so (include/pnp_rccl.h) in a process that never imports
    torch: tests/rccl_native_worker.py."""
    log = tmp_path / "native.log"
    with open(log, "wb") as f:
        p = subprocess.run([sys.executable, os.path.join(HERE, "rccl_native_worker.py")], stdout=f,
                           stderr=subprocess.STDOUT, timeout=110)
    out = log.read_text(errors="replace")
    assert p.returncode == 0, out[-3000:]
    assert "native rccl world-1 exchange ok" in out


@pytest.mark.gpu
@pytest.mark.parametrize("solo", ["1/4", "7/8"])
def test_solo_ordered_loopback_matches_synchronised(tmp_path, solo):
    """bench.py --solo with the loopback enqueued on the library stream (no
    host syncs, as the RCCL exchange: pnp.shard.SoloExchange.ordered) gives
    the same proof bytes as the synchronised loopback (PNP_EXCHANGE_SYNC=1):
    the stream ordering alone carries the exchange dependencies."""
    import json
    root = os.path.dirname(HERE)
    res = {}
    for mode, extra in (("ordered", {}), ("sync", {"PNP_EXCHANGE_SYNC": "1"})):
        env = dict(os.environ, **extra)
        out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--lg", "16", "--solo", solo,
                              "--steps", "2", "--warmup", "1", "--cpu-lg", "0", "--drop-in", "", "--no-verify"],
                             env=env, capture_output=True, text=True, timeout=110, cwd=root)
        assert out.returncode == 0, out.stderr[-3000:]
        res[mode] = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["ordered"]["solo"]["ordered"] is True
    assert res["sync"]["solo"]["ordered"] is False
    assert res["ordered"]["timed_proofs_identical"] and res["sync"]["timed_proofs_identical"]
    assert res["ordered"]["solo"]["proof_sha256"] == res["sync"]["solo"]["proof_sha256"]
