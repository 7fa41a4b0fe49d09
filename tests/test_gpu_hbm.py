"""HBM budget of a proof (abi.cpp hbm_plan / hbm_budget, pnp_hbm_usage):

  * the plan pnp_load_prover_key budgets with is an upper bound of what the
    first proof really allocates (the library's own allocation counter), and
    not a wild one;
  * a budget without room for the optional tables (PNP_HBM_LIMIT) switches the
    copy-constraint groups / the Lagrange-basis key off and the proof bytes do
    not change;
  * a budget without room for the proof fails the first proof after the key
    load with PNP_E_NOMEM and a message naming the bytes, before any work — on
    every rank of a multi-rank run, even
    when only one rank is short (tests/test_shard.py
    test_hbm_short_rank_fails_every_load)."""
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

pytestmark = pytest.mark.gpu

GiB = 1 << 30


def _instance(ctx, lg):
    from bench import Synthetic
    return Synthetic(ctx, lg, 0, seed=2, circuit="merkle")


def _load(ctx, syn):
    ctx.load_prover_key(syn.pk, syn.n, device_ptrs=True)
    ctx.load_commit_key(syn.ck, syn.n, device_ptrs=True)


@pytest.mark.parametrize("lg", [16, 20])
def test_plan_bounds_the_first_proof(lg):
    import pnp
    ctx = pnp.Context(0)
    try:
        syn = _instance(ctx, lg)
        _load(ctx, syn)
        u0 = ctx.hbm_usage()
        plan = u0["mandatory"] + u0["lagrange"] + u0["groups"] + u0["transient"]
        ctx.kernel_timing(True)
        ctx.prove(syn.cs, device_ptrs=True)
        used = ctx.kernel_bytes("wire_groups_used")
        ctx.kernel_timing(False)
        u1 = ctx.hbm_usage()
        grew = u1["peak"] - u0["live"]
        print(f"2^{lg}: plan {plan / GiB:.3f} GiB (mandatory {u0['mandatory'] / GiB:.3f}, lagrange "
              f"{u0['lagrange'] / GiB:.3f}, groups {u0['groups'] / GiB:.3f}, transient {u0['transient'] / GiB:.3f}); "
              f"first proof peak +{grew / GiB:.3f} GiB, held after {u1['live'] / GiB:.3f} GiB")
        assert used == 1  # the groups were built and used, so the plan covered them
        assert grew <= plan, (grew, plan)
        assert plan <= 3 * grew + (256 << 20), (grew, plan)
        # a second proof allocates nothing new
        ctx.prove(syn.cs, device_ptrs=True)
        assert ctx.hbm_usage()["peak"] <= u1["live"] + (64 << 20)
    finally:
        ctx.close()


def test_budget_switches_optional_tables_off(monkeypatch):
    import pnp
    from pnp import abi
    lg = 16
    ctx = pnp.Context(0)
    try:
        syn = _instance(ctx, lg)
        _load(ctx, syn)
        ref = abi.proof_to_bytes(ctx.prove(syn.cs, device_ptrs=True))
    finally:
        ctx.close()
    for keep_lag in (True, False):
        ctx = pnp.Context(0)
        try:
            syn = _instance(ctx, lg)
            _load(ctx, syn)  # (plans with nothing built yet)
            u = ctx.hbm_usage()
            room = u["live"] + u["mandatory"] + u["transient"] + (u["lagrange"] if keep_lag else 0) + (1 << 20)
            monkeypatch.setenv("PNP_HBM_LIMIT", str(room))  # read by the first proof's budget check
            ctx.kernel_timing(True)
            got = abi.proof_to_bytes(ctx.prove(syn.cs, device_ptrs=True))
            groups = ctx.kernel_bytes("wire_groups_used")
            ctx.kernel_timing(False)
            monkeypatch.delenv("PNP_HBM_LIMIT")
            assert got == ref, keep_lag
            assert groups == 0, keep_lag
        finally:
            ctx.close()


def test_budget_refuses_a_proof_that_cannot_fit(monkeypatch):
    import pnp
    ctx = pnp.Context(0)
    try:
        syn = _instance(ctx, 16)
        _load(ctx, syn)
        monkeypatch.setenv("PNP_HBM_LIMIT", "1")
        with pytest.raises(pnp.PnpError, match="PNP_E_NOMEM.*HBM budget"):
            ctx.prove(syn.cs, device_ptrs=True)
        monkeypatch.delenv("PNP_HBM_LIMIT")
        ctx.prove(syn.cs, device_ptrs=True)  # room again: the key is still loaded and proves
    finally:
        ctx.close()


def test_device_srs_reload_keeps_derived_tables():
    """reloading the SAME device-resident SRS (same address, size
    and bytes) keeps the tables derived from it (folded tables, Lagrange
    basis, copy groups); a changed point drops them (their plan parts are
    positive again)."""
    import torch
    import pnp
    from pnp import abi
    ctx = pnp.Context(0)
    try:
        syn = _instance(ctx, 14)
        _load(ctx, syn)
        ref = abi.proof_to_bytes(ctx.prove(syn.cs, device_ptrs=True))
        u = ctx.hbm_usage()
        assert u["lagrange"] == 0 and u["groups"] == 0, u
        ctx.load_commit_key(syn.ck, syn.n, device_ptrs=True)  # same bytes
        u = ctx.hbm_usage()
        assert u["lagrange"] == 0 and u["groups"] == 0, u
        assert abi.proof_to_bytes(ctx.prove(syn.cs, device_ptrs=True)) == ref
        srs = syn.keep["srs"]
        saved = srs[5].clone()
        srs[5] = srs[6]
        torch.cuda.synchronize()
        ctx.load_commit_key(syn.ck, syn.n, device_ptrs=True)  # one point changed
        u = ctx.hbm_usage()
        assert u["lagrange"] > 0, u
        srs[5] = saved
        torch.cuda.synchronize()
        ctx.load_commit_key(syn.ck, syn.n, device_ptrs=True)
        assert abi.proof_to_bytes(ctx.prove(syn.cs, device_ptrs=True)) == ref
    finally:
        ctx.close()


def test_deferred_tables_first_proof(monkeypatch):
    """PNP_DEFER_TABLES=1: the context's first proof commits without the
    optional tables (no Lagrange basis, no copy groups built: their plan bytes
    stay), the second builds and uses them; all three proofs are the same bytes
    as without the switch."""
    import pnp
    from pnp import abi
    lg = 16
    ctx = pnp.Context(0)
    try:
        syn = _instance(ctx, lg)
        _load(ctx, syn)
        ref = abi.proof_to_bytes(ctx.prove(syn.cs, device_ptrs=True))
    finally:
        ctx.close()
    monkeypatch.setenv("PNP_DEFER_TABLES", "1")
    ctx = pnp.Context(0)  # the switch is read when the context is made
    try:
        syn = _instance(ctx, lg)
        _load(ctx, syn)
        proofs, used, lag = [], [], []
        for _ in range(3):
            ctx.kernel_timing(True)
            proofs.append(abi.proof_to_bytes(ctx.prove(syn.cs, device_ptrs=True)))
            used.append(ctx.kernel_bytes("wire_groups_used"))
            ctx.kernel_timing(False)
            lag.append(ctx.hbm_usage()["lagrange"])
        assert used == [0, 1, 1], used
        assert lag[0] > 0 and lag[1] == 0 and lag[2] == 0, lag
        assert proofs == [ref] * 3
    finally:
        ctx.close()
