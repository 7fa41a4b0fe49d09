"""bench.py --solo's loopback exchange (pnp.shard.SoloExchange), CPU: the
ordered gather (decided by the tag on the device, no host read) leaves the
same slots as the synchronised one (decided on the host) for every tagged
message the library sends (include/pnp_plonk.h PNP_EX_TAG_*), at every world
size the bench models."""
import contextlib
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "zprize23-gpu-submission_amd"))


def _exchanges():
    from pnp.shard import SoloExchange

    class Ordered(SoloExchange):
        ordered = True

        def _on_stream(self):
            return contextlib.nullcontext()

    class Synced(SoloExchange):
        ordered = False

        def _on_stream(self):
            return contextlib.nullcontext()

        def _done(self):
            pass

    return SoloExchange, Ordered, Synced


@pytest.mark.parametrize("world", [2, 4, 8])
def test_ordered_loopback_gather_equals_synchronised(world):
    import torch
    Solo, Ordered, Synced = _exchanges()
    # (tag, library words): flags 8, counts world, device id 1, MSM sums B x 24,
    # status 1 or 5, division carry 4, evaluations 4 x 18
    msgs = ((Solo.TAG_T_FLAGS, 8), (Solo.TAG_COUNTS, world), (Solo.TAG_DEVICE, 1), (0x5EC7A111, 48),
            (0x57A7A500, 1), (0x57A7A500, 5), (0xD1FC0001, 4), (0xE7A15000, 72))
    for rank in (0, world - 1):
        for tag, k in msgs:
            w = k + 1
            outs = []
            for cls in (Ordered, Synced):
                e = cls.__new__(cls)
                e.rank, e.world, e.calls, e.gather_bytes = rank, world, 0, 0
                e.buf = torch.zeros(4096, dtype=torch.int64)
                g = torch.Generator().manual_seed(100 * k + world)
                e.buf[rank * w:(rank + 1) * w] = torch.randint(0, 1 << 40, (w,), generator=g)
                e.buf[(rank + 1) * w - 1] = tag
                e.gather(8 * w)
                outs.append(e.buf[: w * world].clone())
            assert torch.equal(outs[0], outs[1]), (world, rank, hex(tag), k)


def test_synchronised_loopback_refuses_untagged_slot():
    import torch
    _, _, Synced = _exchanges()
    e = Synced.__new__(Synced)
    e.rank, e.world, e.calls, e.gather_bytes = 0, 2, 0, 0
    e.buf = torch.zeros(64, dtype=torch.int64)
    with pytest.raises(ValueError, match="untagged"):
        e.gather(64)
