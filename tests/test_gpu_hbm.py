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
        # the first proof goes without the optional tables and starts their
        # background build (context.h deferred tables); a second proof runs
        # while that build is in flight (the proof's working set and
        # the build's scratch live together), sync waits for the build, the
        # third proof uses the tables: the plan must cover all of it
        first = ctx.prove(syn.cs, device_ptrs=True)
        during = ctx.prove(syn.cs, device_ptrs=True)
        from pnp import abi
        assert abi.proof_to_bytes(during) == abi.proof_to_bytes(first)
        ctx.sync()
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
        # a fourth proof allocates nothing new
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
    """Deferred tables (context.h, the default on one GPU): the context's
    first proof commits without the optional tables (no Lagrange basis, no
    copy groups) and starts their build in the background; a proof right
    after it runs beside the build (and goes without them); pnp_commit_evals
    between proofs waits for the basis (it used to fail with "no
    Lagrange-basis key"); once the build is done the proofs use the tables.
    Every proof is the bytes of a context that builds the tables up front
    (PNP_DEFER_TABLES=0)."""
    import torch
    import pnp
    from pnp import abi
    lg = 16
    monkeypatch.setenv("PNP_DEFER_TABLES", "0")
    ctx = pnp.Context(0)  # the switch is read when the context is made
    try:
        syn = _instance(ctx, lg)
        _load(ctx, syn)
        ctx.kernel_timing(True)
        ref = abi.proof_to_bytes(ctx.prove(syn.cs, device_ptrs=True))
        assert ctx.kernel_bytes("wire_groups_used") == 1  # built by the first proof itself
        ctx.kernel_timing(False)
        ev = syn.keep["w_l"]
        evals = torch.zeros((syn.n, 4), dtype=torch.int64, device="cuda")
        evals[: ev.shape[0]] = ev
        torch.cuda.synchronize()
        c_ref = ctx.commit_evals(evals.data_ptr(), syn.n)
    finally:
        ctx.close()
    monkeypatch.delenv("PNP_DEFER_TABLES")
    ctx = pnp.Context(0)
    try:
        syn = _instance(ctx, lg)
        _load(ctx, syn)
        ctx.kernel_timing(True)
        p1 = abi.proof_to_bytes(ctx.prove(syn.cs, device_ptrs=True))
        assert ctx.kernel_bytes("wire_groups_used") == 0
        ctx.kernel_timing(False)
        p2 = abi.proof_to_bytes(ctx.prove(syn.cs, device_ptrs=True))  # beside the build (or after it)
        ev = syn.keep["w_l"]
        evals = torch.zeros((syn.n, 4), dtype=torch.int64, device="cuda")
        evals[: ev.shape[0]] = ev
        torch.cuda.synchronize()
        c = ctx.commit_evals(evals.data_ptr(), syn.n)  # waits for the background basis
        assert (bytes(c.x), bytes(c.y)) == (bytes(c_ref.x), bytes(c_ref.y))
        ctx.sync()
        lag = ctx.hbm_usage()["lagrange"]
        ctx.kernel_timing(True)
        p3 = abi.proof_to_bytes(ctx.prove(syn.cs, device_ptrs=True))
        used = ctx.kernel_bytes("wire_groups_used")
        ctx.kernel_timing(False)
        assert lag == 0 and used == 1, (lag, used)
        assert [p1, p2, p3] == [ref] * 3
    finally:
        ctx.close()


def test_background_build_then_key_load():
    """A key load while the background build runs waits for it (the build
    reads the keys being replaced); an unchanged key keeps the tables, and the
    proofs keep their bytes.  Destroying a context with a build in flight
    stops it at its next kernel."""
    import pnp
    from pnp import abi
    lg = 16
    ctx = pnp.Context(0)
    try:
        syn = _instance(ctx, lg)
        _load(ctx, syn)
        p1 = abi.proof_to_bytes(ctx.prove(syn.cs, device_ptrs=True))  # starts the build
        _load(ctx, syn)                                                # waits for it
        ctx.kernel_timing(True)
        p2 = abi.proof_to_bytes(ctx.prove(syn.cs, device_ptrs=True))
        used = ctx.kernel_bytes("wire_groups_used")
        ctx.kernel_timing(False)
        assert used == 1
        assert p1 == p2
    finally:
        ctx.close()
    ctx = pnp.Context(0)
    syn = _instance(ctx, lg)
    _load(ctx, syn)
    assert abi.proof_to_bytes(ctx.prove(syn.cs, device_ptrs=True)) == p1  # starts a build
    ctx.close()  # stops it


def test_exchange_setters_stop_the_background_build():
    """pnp_set_msm_shard / pnp_set_exchange_v / _a2a change what
    the background build reads (the world, the exchange) and release the table
    it may be writing, so they stop it first.  A world-1 proof starts the
    build, the setters run at once (set_msm_shard(None) calls all three), the
    next proof keeps the bytes, and a later build completes and is used."""
    import pnp
    from pnp import abi
    lg = 16
    ctx = pnp.Context(0)
    try:
        syn = _instance(ctx, lg)
        _load(ctx, syn)
        p1 = abi.proof_to_bytes(ctx.prove(syn.cs, device_ptrs=True))  # starts the build
        ctx.set_msm_shard(None)                                        # stops it
        p2 = abi.proof_to_bytes(ctx.prove(syn.cs, device_ptrs=True))  # (may start another)
        ctx.sync()
        ctx.kernel_timing(True)
        p3 = abi.proof_to_bytes(ctx.prove(syn.cs, device_ptrs=True))
        ctx.sync()
        p4 = abi.proof_to_bytes(ctx.prove(syn.cs, device_ptrs=True))
        used = ctx.kernel_bytes("wire_groups_used")
        ctx.kernel_timing(False)
        assert p1 == p2 == p3 == p4
        assert used >= 1, used
    finally:
        ctx.close()
