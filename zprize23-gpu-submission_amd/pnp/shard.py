"""Multi-GPU gen_proof exchange (include/pnp_plonk.h, pnp_set_msm_shard and
pnp_set_exchange_a2a).

The reference proves on one GPU; SURVEY.md §8(e) maps its multi-GPU story to
sharding the MSMs across the GPUs of a node.  Every rank runs the whole
gen_proof and returns the same ProofC:
  * MSMs: rank r takes a contiguous point range (every window) and the B
    partial sums of a batch meet in one in-place all-gather of B x 192 B
    (`gather`); the same slots carry a few scalars per rank.
  * round 4 (optional, `a2a_bytes` > 0, world | 8): rank r owns 8/world of the
    8n coset blocks for the LDEs and the quotient and one coefficient range of
    everything after; one all-to-all (`alltoall`) moves the inverse block
    transforms into coefficient ranges.
RCCL (backend "nccl") runs both collectives on device buffers over xGMI; gloo
(CPU tests, or several ranks sharing one GPU) goes through host memory.
"""
import ctypes as C

from . import ALLGATHER_FN, ALLTOALL_FN, ALLTOALLV_FN


class WindowExchange:
    """Device buffers and collectives of one rank.

    `buf`: the all-gather slots (world * bytes_per_rank, rank-major).
    `a2a`: the all-to-all buffer, send slots then receive slots."""

    def __init__(self, rank: int, world: int, group=None, device=None,
                 capacity_bytes: int = 1 << 20, a2a_bytes: int = 0, v_bytes: int = 0):
        import torch
        import torch.distributed as dist
        self.rank, self.world, self.group = rank, world, group
        self.buf = torch.zeros(capacity_bytes // 8, dtype=torch.int64, device=device)
        self.a2a = (torch.zeros(a2a_bytes // 8, dtype=torch.int64, device=device)
                    if a2a_bytes and world > 1 else None)
        # bucket-range MSMs (pnp_set_exchange_v): send / receive record buffers
        self.vsend = torch.empty(v_bytes // 8, dtype=torch.int64, device=device) if v_bytes and world > 1 else None
        self.vrecv = torch.empty(v_bytes // 8, dtype=torch.int64, device=device) if v_bytes and world > 1 else None
        self.v_calls = 0
        if self.buf.is_cuda:
            torch.cuda.synchronize()
        self.backend = dist.get_backend(group) if world > 1 else "none"
        self.calls = 0
        self.a2a_calls = 0
        self.error = None
        # the library's stream (pnp.Context.set_msm_shard sets it): RCCL
        # collectives are enqueued behind the library's work on that stream and
        # the library's next work behind them — no host synchronisation
        # (pnp_set_exchange_ordered); PNP_EXCHANGE_SYNC=1 keeps the host syncs
        self.stream = None
        self.cb_seconds = 0.0

    @property
    def ordered(self) -> bool:
        import os
        return (self.backend == "nccl" and self.buf.is_cuda and self.stream is not None
                and os.environ.get("PNP_EXCHANGE_SYNC") != "1")

    def _on_stream(self):
        import contextlib
        import torch
        return torch.cuda.stream(self.stream) if self.ordered else contextlib.nullcontext()

    def gather(self, bytes_per_rank: int) -> None:
        import torch
        import torch.distributed as dist
        if bytes_per_rank % 8 or bytes_per_rank * self.world > self.buf.numel() * 8:
            raise ValueError(f"bad slot size {bytes_per_rank}")
        w = bytes_per_rank // 8
        out = self.buf[: w * self.world]
        mine = out[self.rank * w:(self.rank + 1) * w]
        if self.buf.is_cuda and self.backend == "nccl":
            # RCCL all-gather; the input is a copy of this rank's slot (B x 192 B)
            # rather than a view into the output, so no overlap rule of the
            # torch / RCCL versions at hand can reject it
            with self._on_stream():
                dist.all_gather_into_tensor(out, mine.clone(), group=self.group)
            if not self.ordered:
                torch.cuda.current_stream().synchronize()
        else:
            host_mine = mine.cpu().clone()
            parts = [torch.empty_like(host_mine) for _ in range(self.world)]
            dist.all_gather(parts, host_mine, group=self.group)
            out.copy_(torch.cat(parts))
            if self.buf.is_cuda:
                torch.cuda.current_stream().synchronize()
        self.calls += 1

    def alltoall(self, bytes_per_peer: int) -> None:
        import torch
        import torch.distributed as dist
        if self.a2a is None or bytes_per_peer % 8 or 2 * bytes_per_peer * self.world > self.a2a.numel() * 8:
            raise ValueError(f"bad all-to-all slot size {bytes_per_peer}")
        w = bytes_per_peer // 8
        send = self.a2a[: w * self.world]
        recv = self.a2a[w * self.world: 2 * w * self.world]
        if self.a2a.is_cuda and self.backend == "nccl":
            with self._on_stream():
                dist.all_to_all_single(recv, send, group=self.group)
            if not self.ordered:
                torch.cuda.current_stream().synchronize()
        else:
            # through host memory, one exchange per peer pair (gloo)
            h_send = send.cpu().clone()
            h_recv = torch.empty_like(h_send)
            if self.backend == "gloo":
                dist.all_to_all_single(h_recv, h_send, group=self.group)
            else:
                h_recv.copy_(h_send)
            recv.copy_(h_recv)
            if self.a2a.is_cuda:
                torch.cuda.current_stream().synchronize()
        self.a2a_calls += 1

    def _count_dest(self, send_bytes):
        """bytes this rank sent to each bucket range (the balance of the
        bucket-range split: bench.py reports max / mean)"""
        if not hasattr(self, "v_sent_to") or len(self.v_sent_to) != self.world:
            self.v_sent_to = [0] * self.world
        for d in range(self.world):
            self.v_sent_to[d] += int(send_bytes[d])

    def alltoallv(self, send_bytes, recv_bytes) -> None:
        """Segment s of `vsend` (send_bytes[s] bytes, back to back) goes to rank
        s; what rank s sent lands at sum(recv_bytes[:s]) of `vrecv`."""
        import torch
        import torch.distributed as dist
        self._count_dest(send_bytes)
        ss = [int(b) // 8 for b in send_bytes]
        rs = [int(b) // 8 for b in recv_bytes]
        send = self.vsend[: sum(ss)]
        recv = self.vrecv[: sum(rs)]
        if self.vsend.is_cuda and self.backend == "nccl":
            with self._on_stream():
                dist.all_to_all_single(recv, send, output_split_sizes=rs, input_split_sizes=ss, group=self.group)
            if not self.ordered:
                torch.cuda.current_stream().synchronize()
        else:
            h_recv = torch.empty(sum(rs), dtype=torch.int64)
            dist.all_to_all_single(h_recv, send.cpu(), output_split_sizes=rs, input_split_sizes=ss,
                                   group=self.group)
            recv.copy_(h_recv)
            if self.vsend.is_cuda:
                torch.cuda.current_stream().synchronize()
        self.v_calls += 1

    def _timed(self, fn, *a) -> int:
        import time
        t0 = time.perf_counter()
        try:
            fn(*a)
            return 0
        except Exception as e:  # never unwind through the C++ frames
            self.error = e
            return 1
        finally:
            self.cb_seconds += time.perf_counter() - t0

    def c_alltoallv(self):
        def cb(_user, send_bytes, recv_bytes):
            return self._timed(self.alltoallv, [send_bytes[i] for i in range(self.world)],
                               [recv_bytes[i] for i in range(self.world)])
        return ALLTOALLV_FN(cb)

    def c_callback(self):
        def cb(_user, bytes_per_rank):
            return self._timed(self.gather, int(bytes_per_rank))
        return ALLGATHER_FN(cb)

    def c_alltoall(self):
        def cb(_user, bytes_per_peer):
            return self._timed(self.alltoall, int(bytes_per_peer))
        return ALLTOALL_FN(cb)


class SoloExchange(WindowExchange):
    """One rank of a `world`-GPU proof run ALONE on one GPU (bench.py --solo):
    the library does exactly rank `rank`'s share of the work (its MSM point
    ranges, its round-4 blocks and coefficient range), and the collectives
    are loopbacks (every slot gets this rank's data; the all-to-all returns
    what was sent).  The proof is meaningless; the time is the per-rank
    critical path of the multi-GPU proof without the xGMI transfers, which
    the caller accounts for separately (`calls`, `bytes`)."""

    def __init__(self, rank: int, world: int, device=None, a2a_bytes: int = 0, v_bytes: int = 0):
        import torch
        self.rank, self.world, self.group = rank, world, None
        self.buf = torch.zeros((1 << 20) // 8, dtype=torch.int64, device=device)
        self.a2a = torch.zeros(a2a_bytes // 8, dtype=torch.int64, device=device) if a2a_bytes else None
        self.vsend = torch.empty(v_bytes // 8, dtype=torch.int64, device=device) if v_bytes else None
        self.vrecv = torch.empty(v_bytes // 8, dtype=torch.int64, device=device) if v_bytes else None
        torch.cuda.synchronize()
        self.backend = "loopback"
        self.stream = None
        self.cb_seconds = 0.0
        self.calls = self.a2a_calls = self.v_calls = 0
        self.gather_bytes = self.a2a_bytes_moved = self.v_bytes_moved = 0
        self.error = None

    # Every all-gather slot ends with the library's tag word (include/
    # pnp_plonk.h PNP_EX_TAG_*); the loopback treats two messages specially:
    #  * the quotient chunks' non-zero flags (prover.cpp): the loopback
    #    all-to-all hands this rank its own blocks in every slot, so its t_7 /
    #    t_8 come out non-zero where the real distributed quotient of a
    #    satisfying circuit has them zero; the flags say zero, as every real
    #    rank would, so the rank commits the same 6 chunks as in the real run;
    #  * the bucket-range counts (msm.hip msm_bucket_batch): "rank s" sends
    #    this rank what this rank sends rank s (alltoallv below returns those
    #    segments), so this rank accumulates as many distinct entries as a real
    #    rank, spread over its bucket range like a real rank's.
    #  * the key load's device ids (abi.cpp hbm_budget): the other ranks of a
    #    real run have GPUs of their own, so their slots get other ids (the
    #    rank's HBM budget is its whole GPU, as in the real run).
    TAG_T_FLAGS = 0x7F1A6500
    TAG_COUNTS = 0xB0C4E7C0
    TAG_DEVICE = 0xDE71CE00
    TAGS = (0xB0C4E7C0, 0x5EC7A111, 0x7F1A6500, 0xD1FC0001, 0xE7A15000, 0x57A7A500, 0xDE71CE00)

    @property
    def ordered(self) -> bool:
        """Like the RCCL exchange: the loopback copies are enqueued on the
        library's stream with no host synchronisation (PNP_EXCHANGE_SYNC=1:
        synchronised, as the gloo exchange), so the solo time carries the host
        round trips a real ordered rank pays and no others."""
        import os
        return self.buf.is_cuda and self.stream is not None and os.environ.get("PNP_EXCHANGE_SYNC") != "1"

    def _done(self):
        import torch
        if not self.ordered:
            torch.cuda.current_stream().synchronize()

    def gather(self, bytes_per_rank: int) -> None:
        import torch
        w = bytes_per_rank // 8
        with self._on_stream():
            mine = self.buf[self.rank * w:(self.rank + 1) * w].clone()
            slots = self.buf[: w * self.world].view(self.world, w)
            if not self.ordered:
                tag = int(mine[-1]) & 0xFFFFFFFFFFFFFFFF
                if tag not in self.TAGS:
                    raise ValueError(f"untagged all-gather slot ({bytes_per_rank} B, last word {tag:#x})")
                if tag == self.TAG_T_FLAGS:
                    mine[6:8] = 0
                slots.copy_(mine.expand(self.world, w))
                if tag == self.TAG_COUNTS:
                    slots[:, self.rank] = mine[: self.world]
                if tag == self.TAG_DEVICE:
                    slots[:, 0] += torch.arange(self.world, device=slots.device) - self.rank
            else:
                # the same three cases, decided by the tag on the device (no host
                # read), each only at its slot size (library words + the tag:
                # flags 9, counts world + 1, device ids 2), so a gather costs two
                # or three small kernels as an RCCL gather costs two; the tags
                # themselves are checked by the synchronised mode, which
                # tests/test_gpu_rccl.py requires to give the same proof
                tag = mine[-1]
                if w == 9:
                    mine[6:8] *= (tag != self.TAG_T_FLAGS)
                slots.copy_(mine.expand(self.world, w))
                if w == self.world + 1:
                    slots[:, self.rank] = torch.where(tag == self.TAG_COUNTS, mine[: self.world], slots[:, self.rank])
                if w == 2:
                    slots[:, 0] += (torch.arange(self.world, device=slots.device) - self.rank) * (tag == self.TAG_DEVICE)
        self._done()
        self.calls += 1
        self.gather_bytes += bytes_per_rank * self.world

    def alltoall(self, bytes_per_peer: int) -> None:
        w = bytes_per_peer // 8
        with self._on_stream():
            self.a2a[w * self.world: 2 * w * self.world].copy_(self.a2a[: w * self.world])
        self._done()
        self.a2a_calls += 1
        self.a2a_bytes_moved += bytes_per_peer * (self.world - 1)

    def alltoallv(self, send_bytes, recv_bytes) -> None:
        """Loopback: receive segment s = this rank's send segment s (the count
        exchange above made the sizes agree): distinct entries of this rank's
        points, bucket indices within a range, as many as a real rank gets."""
        self._count_dest(send_bytes)
        ss = [int(b) // 8 for b in send_bytes]
        rs = [int(b) // 8 for b in recv_bytes]
        assert rs == ss, (rs, ss)
        n = sum(ss)
        with self._on_stream():
            self.vrecv[:n].copy_(self.vsend[:n])
        self._done()
        self.v_calls += 1
        self.v_bytes_moved += sum(send_bytes) - send_bytes[self.rank]


def v_bytes_for(lg_n: int, world: int, max_batch: int = 8, slack: float = 2.0) -> int:
    """Capacity of each bucket-range record buffer (pnp_set_exchange_v): the
    8-byte entries of the largest batch (max_batch MSMs x windows x points)
    a rank sends or receives, with `slack` for uneven bucket ranges (a batch
    that still overflows falls back to point ranges)."""
    if world <= 1:
        return 0
    c = 20 if lg_n >= 19 else max(4, lg_n - 3)  # msm_cfg, folded layout
    windows = (256 + c - 1) // c
    per_rank = -(-(1 << lg_n) // world)
    return int(slack * max_batch * windows * per_rank) * 8


def a2a_bytes_for(lg_n: int, world: int) -> int:
    """All-to-all buffer of the distributed round 4 (0 when world does not
    divide 8): send + receive slots of (8/world blocks) x (n/world) Fr."""
    if world <= 1 or 8 % world:
        return 0
    n = 1 << lg_n
    return 2 * world * (8 // world) * (n // world) * 32
