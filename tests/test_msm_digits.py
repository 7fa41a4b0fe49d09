"""The folded MSM's signed digits with the scaled top window (msm_internal.h
MsmCfg::top_sh, msm.hip scalar_digits / msm_build_table), modelled on the
CPU: for every window width the library uses, the keys' magnitudes stay
inside the 2^(c-1) buckets, the weighted sum over the table levels (level k =
2^(c k) P, the top level 2^(c (W-1) - top_sh) P) reproduces the scalar, and
the top window's entries spread over the whole bucket range (so a
bucket-range sharded MSM gives every rank its share: unscaled they all land in
the lowest 2^15 buckets, rank 0's range)."""
import random

import pytest

R = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001


def cfg(c):
    W = (256 + c - 1) // c
    top_bits = 255 - c * (W - 1)
    top_sh = c - 1 - top_bits if top_bits >= 0 and c - 1 - top_bits > 0 else 0
    return W, 1 << (c - 1), top_sh


def digits(s, c):
    """(magnitude, sign) per window as scalar_digits makes them (None: zero)."""
    W, NB, top_sh = cfg(c)
    out, carry = [], 0
    for w in range(W):
        raw = ((s >> (w * c)) & ((1 << c) - 1)) + carry
        if raw > NB:
            mag, carry = (NB << 1) - raw, 1
            out.append((mag, -1) if mag else None)
        else:
            carry = 0
            out.append(((raw << top_sh if w == W - 1 else raw), 1) if raw else None)
    assert carry == 0
    return out


@pytest.mark.parametrize("c", [4, 8, 9, 10, 13, 16, 17, 18, 19, 20])
def test_scaled_top_window_reconstructs(c):
    W, NB, top_sh = cfg(c)
    rng = random.Random(c)
    samples = [0, 1, R - 1, (1 << 254), R - (1 << 200)] + [rng.randrange(R) for _ in range(400)]
    for s in samples:
        acc = 0
        for w, d in enumerate(digits(s, c)):
            if d is None:
                continue
            mag, sign = d
            assert 1 <= mag <= NB, (c, w, mag)
            level = c * w - (top_sh if w == W - 1 else 0)  # table level exponent
            acc += sign * mag * (1 << level)
        assert acc == s, (c, s)


def test_top_window_spreads_over_bucket_ranges():
    c, world = 20, 8
    W, NB, top_sh = cfg(c)
    assert (W, top_sh) == (13, 4)
    rng = random.Random(7)
    per_rank = [0] * world
    for _ in range(20000):
        d = digits(rng.randrange(R), c)[W - 1]
        if d:
            per_rank[(d[0] - 1) * world // NB] += 1
    # no rank's range is overloaded by the top window (r < 0.91 x 2^255: the
    # last range gets less), and over all 13 windows (the other 12 uniform)
    # the ranks' entry counts are within 2% of each other
    avg = sum(per_rank) / world
    assert max(per_rank) < 1.2 * avg, per_rank
    total = [12 * avg + k for k in per_rank]
    assert max(total) < 1.02 * sum(total) / world, total
