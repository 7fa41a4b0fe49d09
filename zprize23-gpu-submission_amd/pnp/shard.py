"""Multi-GPU gen_proof: window-sharded MSM exchange (include/pnp_plonk.h,
pnp_set_msm_shard).

The reference proves on one GPU; SURVEY.md §8(e) maps its multi-GPU story to
sharding the MSM bucket windows across the GPUs of a node.  Every rank runs
the whole (replicated, deterministic) gen_proof pipeline; inside each batched
MSM rank r accumulates and reduces only its contiguous slice of the virtual
windows, writes the slice's window sums (XYZZ, 192 B each) into its slot of a
shared HBM buffer, and this module's callback all-gathers the slots in place.
The exchange is a few KiB per MSM batch, so one RCCL all-gather over xGMI
costs microseconds; gloo (CPU tests, or several ranks sharing one GPU) goes
through host memory.
"""
import ctypes as C

from . import ALLGATHER_FN


class WindowExchange:
    """In-place all-gather of per-rank MSM window-sum slots.

    `buf` is an int64 tensor (HBM when `device` is a GPU) whose first
    world * bytes_per_rank bytes are laid out slot-major; the library writes
    slot `rank` and expects all slots filled after `gather` returns."""

    def __init__(self, rank: int, world: int, group=None, device=None,
                 capacity_bytes: int = 1 << 20):
        import torch
        import torch.distributed as dist
        self.rank, self.world, self.group = rank, world, group
        self.buf = torch.zeros(capacity_bytes // 8, dtype=torch.int64, device=device)
        if self.buf.is_cuda:
            torch.cuda.synchronize()
        self.backend = dist.get_backend(group) if world > 1 else "none"
        self.calls = 0
        self.error = None

    def gather(self, bytes_per_rank: int) -> None:
        import torch
        import torch.distributed as dist
        if bytes_per_rank % 8 or bytes_per_rank * self.world > self.buf.numel() * 8:
            raise ValueError(f"bad slot size {bytes_per_rank}")
        w = bytes_per_rank // 8
        out = self.buf[: w * self.world]
        mine = out[self.rank * w:(self.rank + 1) * w]
        if self.buf.is_cuda and self.backend == "nccl":
            # RCCL in-place all-gather (input is this rank's chunk of the output)
            dist.all_gather_into_tensor(out, mine, group=self.group)
            torch.cuda.current_stream().synchronize()
        else:
            host_mine = mine.cpu().clone()
            parts = [torch.empty_like(host_mine) for _ in range(self.world)]
            dist.all_gather(parts, host_mine, group=self.group)
            out.copy_(torch.cat(parts))
            if self.buf.is_cuda:
                torch.cuda.current_stream().synchronize()
        self.calls += 1

    def c_callback(self):
        def cb(_user, bytes_per_rank):
            try:
                self.gather(int(bytes_per_rank))
                return 0
            except Exception as e:  # never unwind through the C++ frames
                self.error = e
                return 1
        return ALLGATHER_FN(cb)
