"""Which condition makes the multi-rank shard tests crawl?

The 8-rank full-size test crawled (instance generation 4 s -> > 300 s) only
when the pytest parent had run in-process GPU tests before it.  This probe runs
the same multi-rank job (tests/shard_worker.py "full", the HEIGHT=13 Merkle
instance at 2^20: ~10 s when nothing interferes) from a parent process set up
in one of these ways, each in a fresh process, one JSON line each:

  clean8     parent holds no GPU state, 8 ranks        (the baseline)
  clean9     parent holds no GPU state, 9 ranks        (process count alone)
  ctx8       parent holds a HIP context (torch), 8 ranks
  pnp8       parent also holds a pnp context that proved once, 8 ranks
  closed8    as pnp8, but the context is closed before the ranks start
  lo8        parent holds torch + ONE lowest-priority stream that ran a kernel
  norm8      parent holds torch + three normal-priority streams that ran kernels
  hi8        parent holds torch + ONE highest-priority stream that ran a kernel
  low8       parent holds torch + ONE stream at HIP's least priority (ctypes)
  pnpctx8    parent holds torch + a pnp context that did nothing yet
  pnphi8     as pnp8 with the side stream at the highest priority and no
             deferred table build (so no least-priority stream at all)

CRAWL_RANK_QUEUES=Q starts the ranks with GPU_MAX_HW_QUEUES=Q, CRAWL_PARENT_QUEUES=Q
sets it for the parent alone (the ranks keep the box's value).  Every line
carries the peak KFD queue census (sysfs) seen while the ranks ran.

    python tools/crawl_probe.py [config ...]   (default: the first four)

A configuration that passes its time limit (CRAWL_LIMIT, 150 s) is recorded
as crawled, its ranks killed, and the probe stops there unless CRAWL_GO_ON=1
(a crawl is a slow GPU, not a hung one).  The heartbeat of tests/test_shard.py
(CPU, cgroup throttling, HBM free, each rank's last line) goes to
gpurun_out/heartbeat.log while the ranks run."""
import json
import os
import pathlib
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "zprize23-gpu-submission_amd"))

LIMIT = int(os.environ.get("CRAWL_LIMIT", "150"))


def kfd_holders():
    """processes of this user with /dev/kfd open (each is one HWS process)"""
    n = 0
    for p in pathlib.Path("/proc").iterdir():
        if not p.name.isdigit():
            continue
        try:
            if any(os.readlink(f) == "/dev/kfd" for f in (p / "fd").iterdir()):
                n += 1
        except OSError:
            pass
    return n


def run(name, world):
    import test_shard
    import threading
    peak = {"total": 0, "procs": 0, "parent": 0}
    stop = threading.Event()

    def sample():  # the KFD queue census while the ranks live, per GPU
        while not stop.is_set():
            qs = test_shard.kfd_queue_census()
            if sum(qs.values()) > peak["total"]:
                peak.update(total=sum(qs.values()), procs=len(qs), parent=qs.get(os.getpid(), 0),
                            per_process=sorted(qs.values()))
                byg = test_shard.kfd_queue_census_by_gpu()
                # per GPU: each process's queue types (the GPU with the ranks is the busy one)
                peak["by_gpu"] = {g: sorted(",".join(sorted(t)) for t in pq.values()) for g, pq in byg.items()}
            stop.wait(1.0)
    th = threading.Thread(target=sample, daemon=True)
    th.start()
    extra = {"GPU_MAX_HW_QUEUES": os.environ.get("CRAWL_RANK_QUEUES", os.environ.get("CRAWL_QUEUES0", "4"))}
    with open(os.path.join(REPO, "tests", "golden", "merkle_h13_seed1.json")) as f:
        g = json.load(f)
    tmp = pathlib.Path(tempfile.mkdtemp(prefix=f"crawl_{name}_"))
    t0 = time.time()
    ok, err = True, ""
    try:
        test_shard._launch(world, ["full", str(tmp / "p"), str(g["lg"]), str(g["gates"]), str(g["seed"]), "merkle"],
                           tmp, LIMIT, PNP_TEST_MSM_SHARD="points", PNP_EXPECT_BUCKETS="0", **extra)
        for r in range(world):
            if open(tmp / f"p.{r}", "rb").read().hex() != g["proof_hex"]:
                ok, err = False, f"rank {r} proof differs"
    except Exception as e:  # a rank that failed or passed the limit
        ok, err = False, repr(e)[-400:]
    dt = time.time() - t0
    print(json.dumps({"config": name, "ranks_done_s": round(dt, 1), "ok": ok, "error": err[-200:]}), flush=True)
    stop.set()
    th.join()
    lines = {}
    for r in range(world):
        try:
            lines[r] = (tmp / f"rank{r}.log").read_text(errors="replace").strip().splitlines()[-3:]
        except OSError:
            pass
    rec = {"config": name, "ranks": world, "rank_hw_queues_env": extra.get("GPU_MAX_HW_QUEUES"),
           "parent_hw_queues_env": os.environ.get("CRAWL_PARENT_QUEUES"),
           "queue_census_peak": peak, "seconds": round(dt, 1), "ok": ok, "crawled": dt >= LIMIT - 5,
           "kfd_processes_after": kfd_holders(), "error": err, "rank_tail": {0: lines.get(0), world - 1: lines.get(world - 1)}}
    print(json.dumps(rec), flush=True)
    return ok and not rec["crawled"]


def one(c):
    """set this (fresh) process up as configuration c, then run the ranks"""
    if os.environ.get("CRAWL_PARENT_QUEUES"):  # this process only; the ranks get theirs below
        os.environ["GPU_MAX_HW_QUEUES"] = os.environ["CRAWL_PARENT_QUEUES"]
    if c not in ("clean8", "clean9"):
        import torch
        torch.cuda.init()
        x = torch.ones(1 << 20, device="cuda")
        x.add_(1)
        if c in ("lo8", "hi8", "norm8"):
            try:
                lo, hi = torch.cuda.Stream.priority_range()
            except Exception:
                lo, hi = 0, -1
            prios = {"lo8": [lo], "hi8": [hi], "norm8": [0, 0, 0]}[c]
            streams = [torch.cuda.Stream(priority=p) for p in prios]
            for st in streams:
                with torch.cuda.stream(st):
                    x.add_(1)
            globals()["_streams"] = streams
            print(json.dumps({"config": c, "priority_range": [lo, hi], "priorities": prios}), flush=True)
        torch.cuda.synchronize()
    if c == "low8":  # one stream at HIP's LEAST priority (torch's range stops at normal)
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        lo, hi = ctypes.c_int(), ctypes.c_int()
        hip.hipDeviceGetStreamPriorityRange(ctypes.byref(lo), ctypes.byref(hi))
        st = ctypes.c_void_p()
        assert hip.hipStreamCreateWithPriority(ctypes.byref(st), 1, lo) == 0
        assert hip.hipMemsetAsync(ctypes.c_void_p(x.data_ptr()), 0, 1 << 20, st) == 0
        assert hip.hipStreamSynchronize(st) == 0
        globals()["_lo_stream"] = st
        print(json.dumps({"config": c, "hip_priority_range": [lo.value, hi.value], "priority": lo.value}), flush=True)
    if c == "pnphi8":  # the pnp context without a least-priority stream
        os.environ["PNP_SIDE_PRIORITY"] = "hi"
        os.environ["PNP_DEFER_TABLES"] = "0"
    if c == "pnpctx8":  # a pnp context and nothing else (one stream)
        import pnp
        globals()["_keep"] = pnp.Context(0)
    if c in ("pnp8", "closed8", "pnphi8"):
        import pnp
        from pnp_testlib import Inputs
        inp = Inputs(10, 3)
        ctx = pnp.Context(0)
        ctx.load_prover_key(inp.pk, inp.n, device_ptrs=False)
        ctx.load_commit_key(inp.ck, inp.n, device_ptrs=False)
        ctx.prove(inp.circuit, device_ptrs=False)
        ctx.sync()
        if c == "closed8":
            ctx.close()
        else:
            globals()["_keep"] = ctx  # held like a test's context until the process ends
    print(json.dumps({"config": c, "parent_set_up": True}), flush=True)
    return 0 if run(c, 9 if c == "clean9" else 8) else 1


def one_logged(c):
    import traceback
    try:
        return one(c)
    except BaseException:
        print(json.dumps({"config": c, "exception": traceback.format_exc()[-1500:]}), flush=True)
        raise


def main():
    # the ranks' default: this process's own setting before any knob (4 on the box)
    os.environ.setdefault("CRAWL_QUEUES0", os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    if len(sys.argv) > 2 and sys.argv[1] == "--one":
        return one_logged(sys.argv[2])
    configs = sys.argv[1:] or ["clean8", "clean9", "ctx8", "pnp8"]
    for c in configs:
        rc = subprocess.run([sys.executable, "-u", "-X", "faulthandler", os.path.abspath(__file__), "--one", c],
                            timeout=LIMIT + 240).returncode
        print(json.dumps({"config": c, "child_rc": rc}), flush=True)
        if rc and os.environ.get("CRAWL_GO_ON") != "1":
            print(json.dumps({"stopped_after": c}), flush=True)
            return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
