"""CPU model of the accumulation lanes' bucket walk (csrc/msm.hip
next_bucket): after a piece ends at sorted entry k, the bucket holding k is
found by a galloping search over the bucket starts instead of stepping over
empty buckets one load at a time (a lane crossing an MSM with no entries in a
rank's bucket range stepped over 65,536 of them).  The model follows the HIP
code line for line and must agree with the one-by-one walk it replaced."""
import numpy as np
import pytest


def next_bucket(offs, U, a, k):
    """msm.hip next_bucket: start(a) == k, a < U; the last u >= a with
    start(u) <= k, and start(u + 1); plus the loads it issued."""
    lo, hi, step = a, a + 1, 1
    vhi = offs[hi]
    loads = 1
    while vhi <= k:
        lo = hi
        step <<= 1
        hi = lo + step if lo + step < U else U
        vhi = offs[hi]
        loads += 1
    while hi - lo > 1:
        m = (lo + hi) >> 1
        vm = offs[m]
        loads += 1
        if vm <= k:
            lo = m
        else:
            hi, vhi = m, vm
    return lo, vhi, loads


def walk(offs, cur, k):
    """the replaced walk: do { cur++; next = offs[cur + 1]; } while (next == k)"""
    loads = 0
    while True:
        cur += 1
        nxt = offs[cur + 1]
        loads += 1
        if nxt != k:
            return cur, nxt, loads


def bucket_starts(counts):
    return np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)


@pytest.mark.parametrize("seed", range(6))
def test_gallop_equals_walk(seed):
    rng = np.random.default_rng(seed)
    U = int(rng.integers(50, 3000))
    counts = rng.poisson(rng.uniform(0.2, 4), U)
    # long empty runs: whole "MSMs" with no entries, and the last buckets
    for _ in range(3):
        a = int(rng.integers(0, U))
        counts[a:a + int(rng.integers(1, U // 3 + 2))] = 0
    counts[-int(rng.integers(1, 5)):] = 0
    counts[int(rng.integers(0, U))] += 1  # at least one entry
    offs = bucket_starts(counts)
    total = int(offs[U])
    # every piece boundary a lane can meet: each entry k that starts a bucket
    # after the first bucket holding entries
    for cur in range(U):
        nxt = offs[cur + 1]
        if offs[cur] == nxt or nxt >= total:
            continue  # cur empty, or the last non-empty bucket
        k = int(nxt)
        w_cur, w_next, w_loads = walk(offs, cur, k)
        g_cur, g_next, g_loads = next_bucket(offs, U, cur + 1, k)
        assert (g_cur, g_next) == (w_cur, w_next)
        assert offs[g_cur] <= k < offs[g_cur + 1]
        run = w_cur - cur - 1  # empty buckets skipped
        if run == 0:
            assert g_loads == 1  # the common case costs what the walk did
        else:
            assert g_loads <= 2 * (run + 1).bit_length() + 1


def test_whole_empty_msm_costs_log_loads():
    # three MSMs of 65,536 buckets, the middle one empty (rank 7's wire c)
    NB = 1 << 16
    counts = np.ones(3 * NB, dtype=np.int64)
    counts[NB:2 * NB] = 0
    offs = bucket_starts(counts)
    cur, k = NB - 1, int(offs[NB])
    w = walk(offs, cur, k)
    g = next_bucket(offs, len(counts), cur + 1, k)
    assert g[:2] == w[:2] and w[2] == NB + 1 and g[2] <= 35
