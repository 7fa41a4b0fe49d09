"""gen_proof benchmark on MI355X (BASELINE.json metric).

One step = one gen_proof of the HEIGHT=15 Poseidon-Merkle circuit (3,161,924
gates -> domain n = 2^22, quotient on the 8n = 2^25 coset) with the prover
key, SRS and witness already resident in HBM (v2 API, pnp_prove with device
pointers).  Inputs are generated on the GPU (seeded): by default
(--circuit merkle, pnp_synth_merkle) the reference's own circuit — width-3
Poseidon with the plonk-hashing constants, the merkle-tree constraint layout
row for row (checked against tests/merkle_circuit.py), random leaves and
blinding values; --circuit arith (pnp_synth_circuit) is the round-1 stand-in,
a satisfying random arithmetic circuit of the same size.  Prover-key
evaluations = coset LDE of the coefficients; real coset points and Z_H
values; SRS = [tau^i] G.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

N > 1: one process per GPU; all ranks prove the SAME instance together
(DESIGN.md 6): every MSM is split by point ranges (rank r sums points
[r n/N, (r+1) n/N) over all windows; the partial sums meet in one RCCL
all-gather per batch), round 4 is split by coset blocks / coefficient ranges
with one all-to-all, rounds 1-3 and the transcript are replicated.  value =
max over ranks of the per-proof time (strong scaling: one proof regardless of
N).  Rank 0 prints ONE JSON line.  Without WORLD_SIZE in the environment,
`--gpus N` (N > 1) relaunches itself under torch.distributed.run with N ranks
before touching the GPU, and refuses to run when fewer than N GPUs are
visible; a world size different from --gpus is an error.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "zprize23-gpu-submission_amd"))

HEIGHT15_GATES = 3_161_924
REF_SECONDS = (9.543495451 + 9.337866544 + 9.287114947 + 9.309883876) / 4  # TOP-README:16-19
HBM_PEAK_GBS = 8000.0                      # MI355X_MICROARCH.md, spec
R_MOD = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
METRIC = "gen_proof wall-clock (s), HEIGHT=15 Poseidon tree, 1/2/4/8 MI355X + HBM GB/s"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class Synthetic:
    """HEIGHT=15-shaped gen_proof inputs, generated and kept on the GPU."""

    POLYS = ("q_l", "q_r", "q_o", "q_4", "q_c", "q_hl", "q_hr", "q_h4", "q_arith",
             "left_sigma", "right_sigma", "out_sigma", "fourth_sigma")

    def __init__(self, ctx, lg_n: int, gates: int, seed: int, circuit: str = "arith"):
        import torch
        from pnp import abi
        n, N8 = 1 << lg_n, 8 << lg_n
        self.n, self.lg_n, self.seed = n, lg_n, seed
        dev = "cuda"
        keep = self.keep = {}

        def alloc(name, elems, limbs=4):
            t = torch.zeros((elems, limbs), dtype=torch.int64, device=dev)
            torch.cuda.synchronize()  # the zero-fill runs on torch's stream, ours is separate
            keep[name] = t
            return t.data_ptr()

        s = seed * 1000
        sel_in = ("q_l", "q_r", "q_o", "q_4", "q_c", "q_hl", "q_hr", "q_h4")
        ev = {p: alloc(p + "_nevals", n) for p in self.POLYS}
        if circuit == "merkle":
            # the reference's own circuit (pnp_synth_merkle, checked row for row
            # against tests/merkle_circuit.py): HEIGHT = lg - 7 (15 at 2^22),
            # random leaves and blinding values, PI = -root at the last gate
            sys.path.insert(0, os.path.join(REPO, "tests"))
            from poseidon import PoseidonConstants, flat_constants
            height = lg_n - 7
            gates = 193 * ((1 << (height - 1)) - 1) + 5
            w = {name: alloc(name, gates) for name in ("w_l", "w_r", "w_o", "w_4")}
            leaves = alloc("leaves", 1 << (height - 1))
            blind = alloc("blind", 8)
            nodes = alloc("nodes", (1 << (height - 1)) - 1)
            ctx.random_fr(leaves, 1 << (height - 1), s + 1)
            ctx.random_fr(blind, 8, s + 2)
            root = ctx.synth_merkle(height, flat_constants(PoseidonConstants()), leaves, blind, nodes,
                                    [w["w_l"], w["w_r"], w["w_o"], w["w_4"]],
                                    [ev[p] for p in sel_in] + [ev["q_arith"]],
                                    [ev[p] for p in ("left_sigma", "right_sigma", "out_sigma", "fourth_sigma")],
                                    n)
            ctx.sync()
            neg = (-root) % R_MOD
            self.pi = (C.c_uint64 * 4)(*[(neg >> (64 * k)) & (2**64 - 1) for k in range(4)])
            pi_pos = gates - 1
            for name in ("leaves", "blind", "nodes"):
                del keep[name]
            self.height = height
        else:
            # satisfying random arithmetic circuit (pnp_synth_circuit): random a, d
            # and selectors, b_i = a_pi(i) copy cycles, c solved from each gate
            w = {name: alloc(name, gates) for name in ("w_l", "w_r", "w_o", "w_4")}
            ctx.random_fr(w["w_l"], gates, s + 1)
            ctx.random_fr(w["w_4"], gates, s + 4)
            self.pi = (C.c_uint64 * 4)(123456789 + seed, 0, 0, 0)
            pi_pos = 7
            for i, p in enumerate(sel_in):
                ctx.random_fr(ev[p], n, s + 100 + i)
            ctx.synth_circuit([w["w_l"], w["w_r"], w["w_o"], w["w_4"]],
                              [ev[p] for p in sel_in] + [ev["q_arith"]],
                              [ev[p] for p in ("left_sigma", "right_sigma", "out_sigma", "fourth_sigma")],
                              n, gates, pi_pos, list(self.pi))
        self.gates, self.circuit = gates, circuit
        qlk = alloc("q_lookup", gates)
        pk = abi.ProverKeyC()
        for p in self.POLYS:
            c = alloc(p + "_coeffs", n)
            e = alloc(p + "_evals", N8)
            torch.cuda.synchronize()
            ctx.sync()
            keep[p + "_coeffs"].copy_(keep[p + "_nevals"])
            torch.cuda.synchronize()
            ctx.ntt(c, lg_n, inverse=True)        # coefficients of the n-domain evaluations
            ctx.coset_lde8(c, e, lg_n)            # 8n coset evaluations (prover key form)
            ctx.sync()
            setattr(pk, p + "_coeffs", abi.ptr(c))
            setattr(pk, p + "_evals", abi.ptr(e))
            del keep[p + "_nevals"]
        zero8 = alloc("zero8", N8)
        zero_n = alloc("zero_n", n)
        empty = alloc("empty", 1)
        for f in ("q_m_evals", "range_selector_evals", "logic_selector_evals",
                  "fixed_group_add_selector_evals", "variable_group_add_selector_evals",
                  "q_lookup_evals"):
            setattr(pk, f, abi.ptr(zero8))
        for f in ("table1", "table2", "table3", "table4"):
            setattr(pk, f, abi.ptr(zero_n))
        for f in ("q_m_coeffs", "range_selector_coeffs", "logic_selector_coeffs",
                  "fixed_group_add_selector_coeffs", "variable_group_add_selector_coeffs",
                  "q_lookup_coeffs"):
            setattr(pk, f, abi.ptr(empty))
        lin = alloc("linear_evaluations", N8)
        vh = alloc("v_h_coset_8n", N8)
        ctx.coset_consts(vh, lin, lg_n)
        pk.linear_evaluations = abi.ptr(lin)
        pk.v_h_coset_8n = abi.ptr(vh)
        srs = alloc("srs", n, 12)
        tau = alloc("tau", 1)
        ctx.random_fr(tau, 1, s + 999)
        torch.cuda.synchronize()
        tau_l = [int(v) & (2**64 - 1) for v in keep["tau"].cpu().view(-1).tolist()]
        ctx.srs(srs, n, tau_l)
        ctx.sync()
        self.pk = pk
        self.ck = abi.CommitKeyC(powers_of_g=abi.ptr(srs), powers_of_gamma_g=abi.ptr(empty))
        self.cs = abi.CircuitC(n=gates, lookup_len=0, intended_pi_pos=pi_pos, q_lookup=abi.ptr(qlk),
                               pi=C.cast(self.pi, abi.U64P), w_l=abi.ptr(w["w_l"]),
                               w_r=abi.ptr(w["w_r"]), w_o=abi.ptr(w["w_o"]), w_4=abi.ptr(w["w_4"]))


# Roofline of k_accumulate29 (integer-VALU bound): every sorted
# (point, window) entry is one XYZZ mixed addition = 8M + 2S = 10 Fq products;
# the hardware bound is the v_mad_u64_u32 issue rate measured by
# tools/ubench_ops.hip (profiles/r02_ubench_ops.txt: cycles per wave64
# instruction per SIMD) over 288 = 2 x 12 x 12 32-bit multiply-adds per
# 381-bit Montgomery product (the textbook CIOS count; this build's radix-2^29
# product spends 392).  The issue-model ceiling (tools/isa_model.py: 19,761
# SIMD cycles per 64 additions of the compiled code) is kept as a secondary.
FQ_PRODUCTS_PER_MADD = 10
ALG_BYTES_PER_ENTRY = 96 + 4
MADS_PER_FQ_PRODUCT = 288
MADD_ISSUE_CYCLES = 19761
MADS_PER_FR_PRODUCT = 128  # 2 x 8 x 8: a b and m q of a 256-bit Montgomery product in 32-bit limbs
# the radix-4 NTT group's ISA: 1,403 VALU per 4 butterflies, 73%
# of them the 8-limb product's v_mad_u64_u32 / v_addc_co_u32 pairs (~4.4 cycles
# each per wave64, profiles/r02_ubench_ops.txt), the rest ~2.2: ~3.8 on average
# k_quotient29_ on the Merkle path (no q_m, one closed-form PI): issue cycles
# per wave of 64 coset points, tools/isa_model.py on protocol.hip with the
# q_m and pi8 branches removed (4,832 v_mad_u64_u32 of 8,709 VALU)
QUOT29_CYCLES_PER_WAVE = 32434
NTT_VALU_PER_BUTTERFLY = 351
NTT_CYCLES_PER_VALU = 0.73 * 4.4 + 0.27 * 2.2
SIMDS, CLOCK_HZ = 256 * 4, 2.4e9
HELD_CLOCK_GHZ = 2.10  # k_accumulate29 under load (DVFS), PMC clock pass, profiles/r02_pmc_clock.txt
UBENCH_FILE = os.path.join(REPO, "profiles", "r02_ubench_ops.txt")


def quotient_roofline(q_ms, q_n, q_gbs, points, prods, merkle):
    """The quotient kernel's line: VALU-bound (VERDICT r05 asked the same of the
    NTT): ~35 Fr products per coset point against 26-36 B of each of ~26 arrays
    — at 8 TB/s the reads take ~40% of the time the products do.  Fr products
    credited by the prover per launch (the path taken), against the textbook
    256-bit Montgomery peak; the compiled kernel's issue model (Merkle path)
    and the HBM figure beside it."""
    out = {"bound": "valu", "launch_ms": round(q_ms / max(q_n, 1), 3),
           "hbm_achieved_gbs": round(q_gbs, 1), "hbm_peak_gbs": HBM_PEAK_GBS,
           "hbm_frac": round(q_gbs / HBM_PEAK_GBS, 4)}
    if q_ms <= 0 or not prods:  # the generic (non radix-2^29) quotient: no count
        out.update({"achieved": None, "peak": None, "frac": None})
        return out
    s = q_ms / 1e3
    fr_peak = SIMDS * CLOCK_HZ * 64 / mad_cycles() / MADS_PER_FR_PRODUCT
    out.update({"achieved": round(prods / s / 1e9, 2), "peak": round(fr_peak / 1e9, 2),
                "unit": "G Fr-mul/s", "frac": round(prods / s / fr_peak, 4),
                "work": "Fr products per coset point on the launched path (34, + 2 with q_m, + 1 with "
                        "the closed-form PI: prover.cpp) x points / HIP-event launch time",
                "points_per_launch": round(points / max(q_n, 1))})
    if merkle:
        out["issue_model_frac"] = round(points / s / 64 * QUOT29_CYCLES_PER_WAVE / (SIMDS * CLOCK_HZ), 4)
    return out


def mad_cycles():
    """Measured cycles per wave64 v_mad_u64_u32 per SIMD (independent chains)."""
    try:
        with open(UBENCH_FILE) as f:
            for line in f:
                if line.startswith("v_mad_u64_u32(sdst)") and "cyc per wave64" in line:
                    return float(line.split("=")[1].split()[0])
    except OSError:
        pass
    return 4.1  # DESIGN.md 4 (round 1 measurement)


PMC_FILE = os.path.join(REPO, "profiles", "r06_accumulate_traffic.json")
def parallelism_label(world: int) -> str:
    """what the multi-rank proof shards: the MSMs by bucket ranges from
    PNP_MSM_BUCKETS_MIN_WORLD (4) ranks on, else by point ranges (msm.hip);
    round 4 by coset blocks when the world size divides 8 (prover.cpp)"""
    points = (os.environ.get("PNP_MSM_SHARD") == "points"
              or world < int(os.environ.get("PNP_MSM_BUCKETS_MIN_WORLD", "4")))
    label = f"msm-{'point' if points else 'bucket'}-range-shard"
    if 8 % world == 0:
        label += " + round4-block-shard"
    return f"{label} x{world}"


def msm_windows(lg: int) -> int:
    """folded windows of an MSM over 2^lg points (msm.hip msm_cfg; as pnp/shard.py v_bytes_for)"""
    c = 20 if lg >= 19 else (lg - 3 if lg > 7 else 4)
    return (256 + c - 1) // c


def pmc_traffic():
    """HBM bytes per k_accumulate29 launch from the committed rocprofv3 PMC
    passes (FETCH_SIZE and WRITE_SIZE in separate runs of this bench; see
    DESIGN.md 5), or None when absent — PMC counters cannot be read live."""
    try:
        with open(PMC_FILE) as f:
            return json.load(f)["bytes_per_launch"]
    except (OSError, ValueError, KeyError):
        return None


def host_copy(syn):
    """(CircuitC, ProverKeyC, CommitKeyC) over host copies of bench.Synthetic's
    device arrays, as the Rust caller hands them over (prover.rs:727-901), +
    the numpy arrays that keep them alive."""
    import numpy as np
    from pnp import abi
    host = {}

    def hp(p):
        addr = C.cast(p, C.c_void_p).value
        if addr not in host:
            for t in syn.keep.values():
                if t.data_ptr() == addr:
                    host[addr] = np.ascontiguousarray(t.cpu().numpy())
                    break
        return abi.ptr(host[addr].ctypes.data)

    cs = syn.cs
    cs_h = abi.CircuitC(n=cs.n, lookup_len=cs.lookup_len, intended_pi_pos=cs.intended_pi_pos,
                        q_lookup=hp(cs.q_lookup), pi=cs.pi, w_l=hp(cs.w_l), w_r=hp(cs.w_r),
                        w_o=hp(cs.w_o), w_4=hp(cs.w_4))
    pk_h = abi.ProverKeyC()
    for f in abi.PK_FIELDS:
        setattr(pk_h, f, hp(getattr(syn.pk, f)))
    ck_h = abi.CommitKeyC(powers_of_g=hp(syn.ck.powers_of_g), powers_of_gamma_g=hp(syn.ck.powers_of_gamma_g))
    return cs_h, pk_h, ck_h, host


def cgroup_cpu_cap():
    """The CPU bandwidth cap of this process's cgroup (v2 cpu.max, v1
    cfs_quota/period) as (CPUs, the raw setting), or (None, setting)."""
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", None)):
        try:
            with open(path) as f:
                raw = f.read().strip()
        except OSError:
            continue
        if parse is not None:
            q, p = (parse(raw) + ["100000"])[:2]
        else:
            q = raw
            try:
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                    p = f.read().strip()
            except OSError:
                p = "100000"
            raw = f"{q} {p}"
        if q in ("max", "-1"):
            return None, raw
        try:
            return max(1, int(int(q) / int(p))), raw
        except ValueError:
            return None, raw
    return None, None


def host_cpu():
    """The host's CPU model, the CPUs this process may run on and any cgroup
    bandwidth cap on them."""
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = os.cpu_count()
    cap, raw = cgroup_cpu_cap()
    return {"model": model, "nproc": os.cpu_count(), "usable": usable,
            "cgroup_cpu_max": raw, "cgroup_cpus": cap,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
            # every usable core (benches/zprize_bench.rs:58-107),
            # unless the cgroup's bandwidth cap allows fewer to run at once
            "threads": min(usable, cap) if cap else usable}


def cpu_baseline(ctx, lg: int, circuit: str, syn=None, gpu_proof=None):
    """Time the CPU restatement (oracle/, test infrastructure; OpenMP on
    every usable host core, overriding an inherited OMP_NUM_THREADS, capped
    only by the cgroup's CPU bandwidth limit) on one gen_proof of the bench's own
    circuit at n = 2^lg, in the same run as the GPU measurement.
    At the bench's own size (the default, HEIGHT = 15) it proves the SAME
    instance the GPU just proved (`syn`, copied to host memory, not timed) and
    its proof must equal the GPU's timed proof; a smaller lg generates a
    smaller instance of the same circuit.  Rank 0 at N = 1 only, after the
    timed region."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import torch
    from pnp import abi
    from pnp_testlib import oracle
    lib = oracle()
    cpu = host_cpu()
    lib.or_set_num_threads(cpu["threads"])
    own = syn is None or syn.lg_n != lg
    if own:
        syn = Synthetic(ctx, lg, int(HEIGHT15_GATES / (1 << 22) * (1 << lg)), seed=1, circuit=circuit)
        gpu_proof = prove_resident(ctx, syn)
    cs_h, pk_h, ck_h, keep = host_copy(syn)
    if own:
        del syn
    torch.cuda.empty_cache()
    out = abi.ProofC()
    res = {}

    def run():  # ctypes releases the GIL: the main thread reports progress
        t = time.perf_counter()
        res["rc"] = lib.or_gen_proof(C.byref(cs_h), C.byref(pk_h), C.byref(ck_h), C.byref(out))
        res["dt"] = time.perf_counter() - t

    import threading
    th = threading.Thread(target=run)
    t0 = time.perf_counter()
    th.start()
    while th.is_alive():
        th.join(30)
        if th.is_alive():
            log(f"cpu baseline: {time.perf_counter() - t0:.0f} s")
    rc, dt = res.get("rc", -1), res.get("dt", 0.0)
    del keep
    return {"value": round(dt, 3), "unit": f"s per gen_proof at n=2^{lg}",
            "cores": int(lib.or_num_threads()), "kind": "port",
            "host": cpu,
            "sample": (f"one gen_proof of the bench's {circuit} circuit at n=2^{lg}"
                       + (f" (HEIGHT={lg - 7} Poseidon Merkle tree, {syn_gates(lg, circuit)} gates)"
                          if circuit == "merkle" else "")
                       + (", the same instance as the timed GPU proofs" if not own else
                          ", a smaller instance of the same circuit")
                       + "; C restatement of the ZK-Garage prover (oracle/, OpenMP, "
                         f"{int(lib.or_num_threads())} threads on {cpu['model'] or 'the host CPU'}); "
                         "inputs copied to host memory before timing"),
            "equals_gpu_proof": rc == 0 and abi.proof_to_bytes(out) == abi.proof_to_bytes(gpu_proof)}


def syn_gates(lg: int, circuit: str) -> int:
    return 193 * ((1 << (lg - 8)) - 1) + 5 if circuit == "merkle" else int(HEIGHT15_GATES / (1 << 22) * (1 << lg))


def prove_resident(ctx, syn):
    ctx.load_prover_key(syn.pk, syn.n, device_ptrs=True)
    ctx.load_commit_key(syn.ck, syn.n, device_ptrs=True)
    return ctx.prove(syn.cs, device_ptrs=True)


def check_proof(syn, proof, circuit: str):
    """Verify the last timed proof, as the reference harness verifies every
    proof it times (benches/pnp_bench.rs:121-136): the restated verifier
    (oracle/verifier.c, Proof::verify, proof.rs:123-431) with the verifier key
    of the bench's prover key built from the SRS trapdoor ([p(tau)] G), the
    KZG checks decided by the trapdoor and, where oracle/_ref holds the
    reference's blst, by its pairing; and, for the seed-1 instances, the
    bytes against the committed golden ProofC.  Checker only, after the timed
    region."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from pnp import abi
    from pnp_testlib import VK_POLYS, verifier_key_tau, verify, kzg_points, fr_unmont, from_limbs
    t0 = time.perf_counter()
    h = lambda t: np.ascontiguousarray(t.cpu().numpy()).view(np.uint64)
    coeffs = {p: h(syn.keep[p + "_coeffs"]) for p in VK_POLYS if p + "_coeffs" in syn.keep}
    tau = h(syn.keep["tau"])[0]
    vk = verifier_key_tau(coeffs, syn.n, h(syn.keep["srs"])[0], tau)
    pis = [(syn.cs.intended_pi_pos, sum(int(v) << (64 * k) for k, v in enumerate(syn.pi)))]
    out = {"trapdoor": bool(verify(vk, proof, pis, tau))}
    try:
        from test_verifier import _blst, pairing_ok
        blst = _blst()
        if blst is not None:
            rc, pts = kzg_points(vk, proof, pis)
            t = fr_unmont(from_limbs(tau))
            out["blst_pairing"] = bool(rc == 0 and pairing_ok(blst, pts[0], pts[1], t)
                                       and pairing_ok(blst, pts[2], pts[3], t))
    except Exception as e:  # the pairing is a second opinion; the trapdoor decides
        out["blst_pairing_error"] = str(e)
    gname = (f"merkle_h{syn.lg_n - 7}_seed{syn.seed}.json" if circuit == "merkle"
             else f"full_2e{syn.lg_n}_seed{syn.seed}.json")
    gpath = os.path.join(REPO, "tests", "golden", gname)
    if os.path.exists(gpath):
        with open(gpath) as f:
            g = json.load(f)
        if g["gates"] == syn.gates:
            out["golden"] = gname
            out["equals_golden"] = abi.proof_to_bytes(proof).hex() == g["proof_hex"]
    out["verified"] = out["trapdoor"] and out.get("blst_pairing", True) and out.get("equals_golden", True)
    out["seconds"] = round(time.perf_counter() - t0, 2)
    return out


def drop_in(ctx, syn, steps: int, v1: bool):
    """What a drop-in Rust caller pays, measured after the
    headline: (a) v2 pnp_prove with the witness in HOST memory (CircuitC as
    prove_pnp builds it, prover.rs:727-762: ~4 x 3.16 M x 32 B over PCIe,
    inside the timed call); (b) the v1 symbol gen_proof with every key in host
    memory: uploading both keys on every call as the reference does
    (PNP_V1_RELOAD=1, load.cu:311-358; the folded SRS table is kept when the
    uploaded SRS is unchanged), the default (every word of both keys hashed on
    the host each call, a key uploaded only when its content changed), and
    PNP_V1_REUSE=1 (resident keys reused by a sampled fingerprint).  Not
    `value`: the headline has inputs already in HBM."""
    import torch
    from pnp import abi
    cs_h, pk_h, ck_h, keep = host_copy(syn)
    out = {}
    ctx.prove(cs_h, device_ptrs=False)
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.prove(cs_h, device_ptrs=False)
    ctx.sync()
    out["v2_host_witness_s"] = round((time.perf_counter() - t0) / steps, 4)
    out["v2_host_witness_inputs_ms"] = round(dict(ctx.stage_times()).get("inputs", 0.0), 2)
    if v1:
        lib = ctx.lib
        ref = abi.proof_to_bytes(ctx.prove(syn.cs, device_ptrs=True))
        same = True
        # The v1 symbol's own context is cold here, but NOT the process: HIP is
        # initialised and the code objects are loaded by the v2 proofs above
        # (the process-cold call, one proof per fresh process as the reference
        # driver makes it, is tools/cold_call.py's v1_process_cold_s).  Its
        # first call hashes and uploads both keys and proves without the
        # optional tables, which then build in the background (context.h);
        # the next calls run beside that build.  Then the steady state of each
        # key mode once the build is done
        cold = []
        for _ in range(3):
            t0 = time.perf_counter()
            p = lib.gen_proof(cs_h, pk_h, ck_h)
            cold.append(round(time.perf_counter() - t0, 3))
            same &= abi.proof_to_bytes(p) == ref
        out["v1_context_cold_calls_s"] = cold
        t0 = time.perf_counter()
        ctx.lib.pnp_sync(C.c_void_p(lib.pnp_v1_context()))
        out["v1_background_build_left_s"] = round(time.perf_counter() - t0, 3)
        # reload: upload both keys every call (the reference's load.cu:311-358);
        # hash (the default): every word of both keys hashed on the host, an
        # unchanged key not uploaded again; reuse: the sampled fingerprint
        for mode in ("hash", "reload", "reuse"):
            os.environ.pop("PNP_V1_RELOAD", None)
            if mode == "reload":
                os.environ["PNP_V1_RELOAD"] = "1"
            if mode == "reuse":
                os.environ["PNP_V1_REUSE"] = "1"
            t0 = time.perf_counter()
            p = lib.gen_proof(cs_h, pk_h, ck_h)
            out[f"v1_{mode}_first_call_s"] = round(time.perf_counter() - t0, 3)
            same &= abi.proof_to_bytes(p) == ref
            t0 = time.perf_counter()
            for _ in range(steps):
                p = lib.gen_proof(cs_h, pk_h, ck_h)
            out[f"v1_{mode}_gen_proof_s"] = round((time.perf_counter() - t0) / steps, 4)
            same &= abi.proof_to_bytes(p) == ref
        os.environ.pop("PNP_V1_REUSE", None)
        os.environ.pop("PNP_V1_RELOAD", None)
        out["v1_equals_v2"] = same
    del keep
    torch.cuda.synchronize()
    return out


NTT_TRAFFIC_FILE = os.path.join(REPO, "profiles", "r05_ntt_traffic.json")


def op_traffic(path, key):
    """HBM bytes per call of an operator line from a committed rocprofv3 PMC
    summary (FETCH_SIZE x 2 per the gfx950 calibration + WRITE_SIZE, separate
    passes), or None."""
    try:
        with open(path) as f:
            return json.load(f)[key]
    except (OSError, ValueError, KeyError):
        return None


def bench_ntt(ctx, lg: int, steps: int, warmup: int, verify: bool):
    """BASELINE config 2: natural-order radix-2 NTT / iNTT of 2^lg Montgomery
    Fr (pnp_ntt = the reference's Ntt / Intt, zksnark_ntt.cu:74-92 with
    arkworks semantics).  A batch of distinct vectors (>= 16 and >= 1 GiB in
    all, so the 256 MiB MALL cannot hold them) is transformed forward then
    inverse in turn; each call is timed with HIP events on the library stream
    (kernel_stats "ntt").  Algorithmic bytes: 2 x 32 B per
    element per transform.  Checked against the CPU restatement on the first
    vector (forward, then the inverse round trip)."""
    import numpy as np
    import torch
    n = 1 << lg
    batch = max(16, (1 << 30) // (32 * n))
    vecs = torch.empty((batch, n, 4), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    for b in range(batch):
        ctx.random_fr(vecs[b].data_ptr(), n, 1000 + b)  # seed 1 family
    ctx.sync()
    x0 = np.ascontiguousarray(vecs[0].cpu().numpy()).view(np.uint64).copy()
    for _ in range(warmup):
        for b in range(batch):
            ctx.ntt(vecs[b].data_ptr(), lg, inverse=False)
            ctx.ntt(vecs[b].data_ptr(), lg, inverse=True)
    ctx.sync()
    ctx.kernel_timing(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        for b in range(batch):
            ctx.ntt(vecs[b].data_ptr(), lg, inverse=False)
        for b in range(batch):
            ctx.ntt(vecs[b].data_ptr(), lg, inverse=True)
    ctx.sync()
    wall = time.perf_counter() - t0
    ms, calls = ctx.kernel_stats("ntt")
    alg = ctx.kernel_bytes("ntt")
    ctx.kernel_timing(False)
    gbs = alg / (ms / 1e3) / 1e9
    per_call = ms / calls
    traffic = op_traffic(NTT_TRAFFIC_FILE, f"bytes_per_call_lg{lg}")
    # VALU roofline (the transform is integer-VALU bound, not
    # HBM-bound; DESIGN.md 7 "The NTT, measured"): the twiddle products done,
    # n/2 (lg - 1) per transform (the half-size-1 level multiplies by 1 and
    # skips the product; the iNTT's n^-1 scaling is not credited), against the
    # textbook peak of 256-bit Montgomery products: 2 x 8 x 8 = 128 32-bit
    # multiply-adds each at the measured v_mad_u64_u32 issue rate.  The HBM
    # figure stays beside it (hbm_frac)
    prods = (n // 2) * (lg - 1) * calls
    fr_rate = prods / (ms / 1e3)
    fr_peak = SIMDS * CLOCK_HZ * 64 / mad_cycles() / MADS_PER_FR_PRODUCT
    bfly_rate = (n // 2) * lg * calls / (ms / 1e3)
    out = {"metric": f"NTT/iNTT 2^{lg} over BLS12-381 Fr (BASELINE config 2): HBM throughput",
           "value": round(gbs, 1), "unit": "GB/s", "n_gpus": 1, "steps": steps, "warmup": warmup,
           "ms_per_step": round(wall * 1e3 / steps, 3), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "u64", "data": "synthetic",
           "config": {"workload": f"natural-order NTT then iNTT of {batch} distinct 2^{lg}-element Fr vectors "
                                  f"per step ({batch * n * 32 / 2**30:.2f} GiB, beyond the 256 MiB MALL)",
                      "domain_log2": lg, "batch": batch, "op": "ntt"},
           "ms_per_transform": round(per_call, 4),
           "roofline": {"bound": "valu", "kernel": "pnp_ntt (k_ntt_pass4 passes + k_bitrev_tiles)",
                        "achieved": round(fr_rate / 1e9, 2), "peak": round(fr_peak / 1e9, 2),
                        "unit": "G Fr-mul/s", "frac": round(fr_rate / fr_peak, 4),
                        "traffic": traffic,
                        "traffic_over_algorithmic": round(traffic / (64 * n), 3) if traffic else None,
                        "work": f"n/2 (lg - 1) twiddle products per transform / HIP-event time per pnp_ntt "
                                f"call on the library stream; peak = {SIMDS} SIMDs x {CLOCK_HZ / 1e9} GHz x 64 "
                                f"lanes / {mad_cycles()} cycles per v_mad_u64_u32 / {MADS_PER_FR_PRODUCT} "
                                "multiply-adds per 256-bit Montgomery product",
                        "butterflies_per_s": round(bfly_rate / 1e9, 2),
                        "valu_per_butterfly_isa": NTT_VALU_PER_BUTTERFLY,
                        "issue_model_frac": round(bfly_rate * NTT_VALU_PER_BUTTERFLY * NTT_CYCLES_PER_VALU
                                                  / (SIMDS * CLOCK_HZ * 64), 4),
                        "hbm_achieved_gbs": round(gbs, 1), "hbm_peak_gbs": HBM_PEAK_GBS,
                        "hbm_frac": round(gbs / HBM_PEAK_GBS, 4),
                        "hbm_work": "2 x 32 B per element per transform (one read, one write: SURVEY 8(d))",
                        "launches": calls}}
    if verify:
        lib = __import__("pnp_testlib").oracle()
        from pnp_testlib import vp
        exp = x0.copy()
        t = time.perf_counter()
        lib.or_ntt(vp(exp), lg, 0, 0)
        cpu_s = time.perf_counter() - t
        d = torch.from_numpy(x0.view(np.int64).copy()).cuda()
        torch.cuda.synchronize()
        ctx.ntt(d.data_ptr(), lg, inverse=False)
        ctx.sync()
        fwd_ok = bool((np.ascontiguousarray(d.cpu().numpy()).view(np.uint64) == exp).all())
        ctx.ntt(d.data_ptr(), lg, inverse=True)
        ctx.sync()
        back_ok = bool((np.ascontiguousarray(d.cpu().numpy()).view(np.uint64) == x0).all())
        out["verified"] = fwd_ok and back_ok
        out["verification"] = {"forward_equals_oracle": fwd_ok, "inverse_round_trip": back_ok}
        cpu = host_cpu()
        out["cpu_baseline"] = {"value": round(n * 64 / cpu_s / 1e9, 3), "unit": "GB/s",
                               "cores": int(lib.or_num_threads()), "kind": "port",
                               "seconds": round(cpu_s, 4), "host": cpu,
                               "sample": f"one forward 2^{lg} NTT of the first vector by the C restatement "
                                         f"(oracle/poly.c or_ntt, radix-2, one thread per butterfly loop)"}
    return out


def bench_msm(ctx, lg: int, steps: int, warmup: int, verify: bool, world: int, rank: int):
    """BASELINE config 3: one 2^lg Pippenger MSM on BLS12-381 G1 against the
    resident commit key (pnp_commit_ck, the folded c = 20 layout gen_proof
    uses; sharded by bucket or point ranges when world > 1), points
    [tau^i] G, scalars uniform Fr (seed 2).  Timed per call with HIP events
    (kernel_stats "msm"); the accumulation's mixed additions counted on the
    device as in the proof line.  Checked against the CPU restatement's MSM
    over the same points and scalars (rank 0)."""
    import numpy as np
    import torch
    n = 1 << lg
    srs = torch.empty((n, 12), dtype=torch.int64, device="cuda")
    tau = torch.empty((1, 4), dtype=torch.int64, device="cuda")
    sc = torch.empty((n, 4), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    ctx.random_fr(tau.data_ptr(), 1, 2999)
    ctx.random_fr(sc.data_ptr(), n, 2)
    ctx.sync()
    ctx.srs(srs.data_ptr(), n, [int(v) & (2**64 - 1) for v in tau.cpu().view(-1).tolist()])
    ctx.sync()
    from pnp import abi
    ctx.load_commit_key(abi.CommitKeyC(powers_of_g=abi.ptr(srs.data_ptr()), powers_of_gamma_g=abi.ptr(srs.data_ptr())),
                        n, device_ptrs=True)
    for _ in range(max(warmup, 1)):  # (the first call builds the folded table)
        ctx.commit_ck(sc.data_ptr(), n)
    ctx.sync()
    ctx.kernel_timing(True)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        c = ctx.commit_ck(sc.data_ptr(), n)
    ctx.sync()
    wall = time.perf_counter() - t0
    ms, calls = ctx.kernel_stats("msm")
    acc_ms, acc_n = ctx.kernel_stats("msm_accumulate")
    madds = ctx.kernel_bytes("msm_madds")
    ctx.kernel_timing(False)
    if world > 1:
        import torch.distributed as dist
        dev = "cuda" if os.environ.get("PNP_BENCH_BACKEND", "nccl") == "nccl" else "cpu"  # (gloo rehearsal)
        t = torch.tensor([wall, ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall, ms = (float(v) for v in t.tolist())
    per = ms / calls
    mad_rate = SIMDS * CLOCK_HZ * 64 / mad_cycles()
    fq_peak = mad_rate / MADS_PER_FQ_PRODUCT
    fq_msm = madds * FQ_PRODUCTS_PER_MADD / (ms / 1e3)            # over the whole MSM time
    fq_acc = madds * FQ_PRODUCTS_PER_MADD / (acc_ms / 1e3) if acc_ms else 0.0
    gbs = n * 128 / (per / 1e3) / 1e9
    out = {"metric": f"Pippenger MSM 2^{lg} on BLS12-381 G1 (BASELINE config 3): time per MSM",
           "value": round(per, 3), "unit": "ms", "n_gpus": world, "steps": steps, "warmup": warmup,
           "ms_per_step": round(wall * 1e3 / steps, 3), "higher_is_better": False, "scaling": "strong",
           "vs_baseline": None, "dtype": "u64", "data": "synthetic",
           "config": {"workload": f"one 2^{lg}-point MSM: points [tau^i] G (resident folded table, c = 20), "
                                  f"uniform Montgomery Fr scalars (seed 2)", "domain_log2": lg, "op": "msm",
                      "parallelism": parallelism_label(world) if world > 1 else "single"},
           "gbs": round(gbs, 1), "gbs_basis": "n (96 + 32) B (every point and scalar once, SURVEY 8(d)) / MSM time",
           "fq_mul_per_s": round(fq_msm / 1e9, 2),
           "roofline": {"bound": "valu", "kernel": "k_accumulate29 (MSM bucket accumulation)",
                        "achieved": round(fq_acc / 1e9, 2), "peak": round(fq_peak / 1e9, 2), "unit": "G Fq-mul/s",
                        "frac": round(fq_acc / fq_peak, 4), "traffic": None,
                        "work": "mixed additions counted on the device x 10 Fq products / summed "
                                "k_accumulate29 launch time (HIP events)",
                        "launch_ms": round(acc_ms / max(acc_n, 1), 3),
                        "madds_per_msm": round(madds / steps),
                        "whole_msm_frac": round(fq_msm / fq_peak, 4)}}
    if verify and rank == 0:
        from pnp_testlib import oracle, vp
        lib = oracle()
        cpu = host_cpu()
        lib.or_set_num_threads(cpu["threads"])
        pts = np.ascontiguousarray(srs.cpu().numpy()).view(np.uint64)
        sch = np.ascontiguousarray(sc.cpu().numpy()).view(np.uint64)
        exp = np.zeros(12, dtype=np.uint64)
        t = time.perf_counter()
        lib.or_commit(vp(pts), vp(sch), n, vp(exp))
        cpu_s = time.perf_counter() - t
        got = np.array(list(c.x) + list(c.y), dtype=np.uint64)
        out["verified"] = bool((got == exp).all())
        out["cpu_baseline"] = {"value": round(cpu_s * 1e3, 1), "unit": "ms", "cores": int(lib.or_num_threads()),
                               "kind": "port", "host": cpu,
                               "sample": f"the same 2^{lg}-point MSM by the C restatement (oracle/g1.c "
                                         "or_commit: Jacobian Pippenger, OpenMP over windows)"}
    return out


def relaunch(n: int) -> int:
    """Start N ranks (one per GPU) under torch.distributed.run as a CHILD
    process; this process never initialises the GPU (device_count() does not
    on this image)."""
    import subprocess
    import torch
    have = torch.cuda.device_count()
    if have < n:
        log(f"bench: --gpus {n} but only {have} GPU(s) visible")
        return 2
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)]
    return subprocess.call(cmd + sys.argv[1:])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--lg", type=int, default=22, help="log2 domain (22 = HEIGHT 15)")
    ap.add_argument("--gates", type=int, default=HEIGHT15_GATES)
    ap.add_argument("--circuit", default="merkle", choices=("merkle", "arith"),
                    help="merkle: the reference's Poseidon Merkle circuit (HEIGHT = lg - 7); "
                         "arith: a random satisfying arithmetic circuit of --gates gates")
    ap.add_argument("--cpu-lg", type=int, default=22,
                    help="CPU baseline size (default: the bench's own HEIGHT=15 instance, ~150 s on 16 "
                         "host threads); 0 = skip")
    ap.add_argument("--no-verify", action="store_true", help="skip the proof check after the timed region")
    ap.add_argument("--solo", default="", metavar="R/W",
                    help="time rank R's share of a W-GPU proof alone on this GPU (loopback exchanges, "
                         "proof discarded): the per-rank critical path of the multi-GPU bench")
    ap.add_argument("--stages", action="store_true", help="print per-stage ms to stderr")
    ap.add_argument("--drop-in", default="v1", choices=("", "v2", "v1"),
                    help="also time the host-witness v2 call ('v2') and the v1 symbol ('v1')")
    ap.add_argument("--op", default="proof", choices=("proof", "ntt", "msm"),
                    help="proof: the headline gen_proof; ntt / msm: the operator lines of BASELINE configs "
                         "2 and 3 (python bench.py --op ntt --lg 20; --op msm --lg 22 [--gpus N])")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return relaunch(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"bench: WORLD_SIZE={world} but --gpus {args.gpus}")
        return 2
    # The v1 symbol as the reference driver calls it, one proof per fresh
    # process (merkle-tree/src/main.rs:102-103): measured first, while this
    # process has made no GPU call (a process that has done GPU work beside
    # the children would share the GPU with them), by
    # tools/cold_call.py's producer and cold children
    cold = None
    if (world == 1 and args.op == "proof" and args.drop_in == "v1" and not args.solo
            and args.circuit == "merkle" and os.environ.get("PNP_BENCH_COLD", "1") != "0"):
        sys.path.insert(0, os.path.join(REPO, "tools"))
        try:
            import cold_call
            cold = cold_call.measure(args.lg, 3, seed=1, log=log)
        except Exception as e:  # reported, never fatal to the headline
            cold = {"v1_process_cold_error": repr(e)}
    import torch
    import torch.distributed as dist
    # PNP_BENCH_BACKEND=gloo: rehearsal of the multi-rank bench on fewer GPUs
    # than ranks (ranks share devices round-robin, exchanges through host
    # memory); the real run is RCCL, one rank per GPU
    backend = os.environ.get("PNP_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    import pnp

    ctx = pnp.Context(local)
    gates = min(args.gates, 1 << args.lg)
    t0 = time.perf_counter()
    solo = None
    # MSM sharding: bucket ranges (default) or point ranges (PNP_MSM_SHARD=points)
    from pnp.shard import v_bytes_for
    vb = (lambda w: 0) if os.environ.get("PNP_MSM_SHARD") == "points" else (lambda w: v_bytes_for(args.lg, w))
    ex = None
    if world > 1:  # sharded MSMs + distributed round 4, exchanges over RCCL
        from pnp.shard import WindowExchange, a2a_bytes_for
        ex = WindowExchange(rank, world, device=torch.device("cuda", local),
                            a2a_bytes=a2a_bytes_for(args.lg, world), v_bytes=vb(world))
        ctx.set_msm_shard(ex)
    elif args.solo:
        from pnp.shard import SoloExchange, a2a_bytes_for
        sr, sw = (int(v) for v in args.solo.split("/"))
        solo = SoloExchange(sr, sw, device=torch.device("cuda", local), a2a_bytes=a2a_bytes_for(args.lg, sw),
                            v_bytes=vb(sw))
        ctx.set_msm_shard(solo)
        args.no_verify, args.drop_in, args.cpu_lg = True, "", 0
    if args.op != "proof":
        if args.op == "ntt" and world > 1:
            log("bench: --op ntt runs on one GPU")
            return 2
        sys.path.insert(0, os.path.join(REPO, "tests"))
        res = (bench_ntt(ctx, args.lg, args.steps, args.warmup, not args.no_verify) if args.op == "ntt" else
               bench_msm(ctx, args.lg, args.steps, args.warmup, not args.no_verify, world, rank))
        if rank == 0:
            print(json.dumps(res), flush=True)
        ctx.close()
        if world > 1:
            dist.destroy_process_group()
        return 0 if res.get("verified", True) else 3
    syn = Synthetic(ctx, args.lg, gates, seed=1, circuit=args.circuit)  # same instance on every rank
    gates = syn.gates
    ctx.load_prover_key(syn.pk, syn.n, device_ptrs=True)
    ctx.load_commit_key(syn.ck, syn.n, device_ptrs=True)
    log(f"[rank {rank}] synthetic inputs + key load: {time.perf_counter() - t0:.1f}s")

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        ctx.prove(syn.cs, device_ptrs=True)
    ctx.kernel_timing(True)
    barrier()
    torch.cuda.synchronize()
    ctx.sync()
    xc = ex if ex is not None else solo
    cb_counts = lambda: ((xc.calls, xc.a2a_calls, getattr(xc, "v_calls", 0), xc.cb_seconds) if xc else (0, 0, 0, 0.0))
    cb0 = cb_counts()
    t0 = time.perf_counter()
    proofs = []
    for _ in range(args.steps):
        proofs.append(ctx.prove(syn.cs, device_ptrs=True))
    ctx.sync()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    # exchange callbacks of the timed proofs only (the warmup's first proof
    # also sizes the fixed slots on the variable path)
    cb1 = cb_counts()
    timed_cb = {"allgathers": (cb1[0] - cb0[0]) / args.steps, "alltoalls": (cb1[1] - cb0[1]) / args.steps,
                "bucket_alltoallvs": (cb1[2] - cb0[2]) / args.steps,
                "callbacks": (cb1[0] + cb1[1] + cb1[2] - cb0[0] - cb0[1] - cb0[2]) / args.steps,
                "callback_ms": 1e3 * (cb1[3] - cb0[3]) / args.steps}
    stages = ctx.stage_times()
    from pnp import abi
    proof = proofs[-1]
    # every timed proof must be the same (the reference harness checks each
    # proof it times, benches/pnp_bench.rs:124-135; the instance is fixed and
    # the prover deterministic, so all equal the first, which is verified below)
    all_equal = all(abi.proof_to_bytes(p) == abi.proof_to_bytes(proofs[0]) for p in proofs)
    acc_ms, acc_n = ctx.kernel_stats("msm_accumulate")
    entries = ctx.kernel_bytes("msm_entries")          # real sorted entries, counted on the device
    madds = ctx.kernel_bytes("msm_madds")              # real mixed additions (entries - fresh pieces)
    dense = ctx.kernel_bytes("msm_entries_dense")      # the dense bound (MSMs x windows x points)
    q_ms, q_n = ctx.kernel_stats("quotient")
    q_bytes = ctx.kernel_bytes("quotient")
    q_points, q_prods = ctx.kernel_bytes("quotient_points"), ctx.kernel_bytes("quotient_fr_products")
    redo_lanes = ctx.kernel_bytes("msm_redo_lanes")
    exact_fallbacks = ctx.kernel_bytes("msm_exact_fallback")
    # bucket-range exchange (world > 1 or --solo): batches moved through the
    # fixed slots, slotted batches redone after an overflow, and the records
    # this rank sent to its busiest bucket range over the mean (the balance)
    slot_batches = ctx.kernel_bytes("msm_slot_batches")
    slot_overflows = ctx.kernel_bytes("msm_slot_overflows")
    dest_max, dest_sum = ctx.kernel_bytes("msm_dest_max"), ctx.kernel_bytes("msm_dest_sum")
    # the whole proof's algorithmic HBM bytes: the
    # prover's per-op credits (minimal reads + writes of every transform, pass
    # and gather), the MSMs' scalars, and 100 B per device-counted sorted entry
    proof_bytes = (ctx.kernel_bytes("proof_alg_bytes") + ctx.kernel_bytes("msm_scalar_bytes")
                   + entries * ALG_BYTES_PER_ENTRY) / args.steps
    ctx.kernel_timing(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    per_proof = elapsed / args.steps
    if args.stages or rank == 0:
        log("stages (ms): " + ", ".join(f"{k}={v:.1f}" for k, v in stages))
        log(f"msm_accumulate: {acc_n} launches, {acc_ms / max(acc_n, 1):.3f} ms avg; "
            f"quotient: {q_n} launches, {q_ms / max(q_n, 1):.3f} ms avg")
    if rank == 0:
        acc_avg_s = acc_ms / max(acc_n, 1) / 1e3
        acc_s = acc_ms / 1e3
        # the dominant kernel's real work: mixed additions counted on the device
        # from the bucket starts of every timed launch (k_count_pieces), per
        # second of its launches (HIP events on the library stream)
        madds_per_s = madds / acc_s if acc_s > 0 else 0.0
        valu_peak = SIMDS * CLOCK_HZ * 64 / MADD_ISSUE_CYCLES
        mad_rate = SIMDS * CLOCK_HZ * 64 / mad_cycles()          # v_mad_u64_u32 / s
        fq_peak = mad_rate / MADS_PER_FQ_PRODUCT                 # Fq products / s
        fq_achieved = madds_per_s * FQ_PRODUCTS_PER_MADD
        # algorithmic bytes: each sorted entry gathers one affine point (96 B)
        # and reads its 4-B index (the reference's per-entry model,
        # pippenger.cuh:147-223)
        alg_per_launch = entries * ALG_BYTES_PER_ENTRY / max(acc_n, 1)
        achieved = entries * ALG_BYTES_PER_ENTRY / acc_s / 1e9 if acc_s > 0 else 0.0
        # the PMC traffic was measured on the default single-GPU workload only
        traffic = pmc_traffic() if (world == 1 and not solo and args.lg == 22 and args.circuit == "merkle") else None
        q_gbs = q_bytes / (q_ms / 1e3) / 1e9 if q_ms > 0 else 0.0
        held = madds_per_s / (valu_peak * HELD_CLOCK_GHZ * 1e9 / CLOCK_HZ)
        if held > 1.0:
            log(f"bench: WARNING k_accumulate29 at {held:.3f} of its issue ceiling at the held clock: "
                "the work count is too high")
        out = {
            "metric": METRIC,
            "value": round(per_proof, 4),
            "unit": "s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(per_proof * 1e3, 2),
            "higher_is_better": False,
            "scaling": "strong",
            "vs_baseline": round(per_proof / REF_SECONDS, 4) if args.lg == 22 else None,
            "dtype": "u64",
            "data": "synthetic",
            "config": {"workload": (f"HEIGHT={syn.height} Poseidon Merkle-tree circuit (the reference's "
                                    f"merkle-tree layout, random leaves)" if args.circuit == "merkle" else
                                    f"random satisfying arithmetic circuit of the HEIGHT=15 size")
                                   + f" gen_proof: {gates} gates, domain 2^{args.lg}, "
                                   f"quotient on 2^{args.lg + 3} coset, pk+SRS+witness HBM-resident",
                       "circuit": args.circuit, "domain_log2": args.lg, "gates": gates,
                       "parallelism": (parallelism_label(world) if world > 1 else
                                       f"solo rank {solo.rank} of {solo.world} (loopback exchanges, "
                                       f"proof discarded)" if solo else "single")},
            "timed_proofs_identical": all_equal,
            "roofline": {"bound": "valu", "kernel": "k_accumulate29 (MSM bucket accumulation)",
                         "achieved": round(fq_achieved / 1e9, 2), "peak": round(fq_peak / 1e9, 2),
                         "unit": "G Fq-mul/s", "frac": round(fq_achieved / fq_peak, 4),
                         "traffic": traffic,
                         "traffic_over_algorithmic": (round(traffic / alg_per_launch, 3)
                                                      if traffic and alg_per_launch else None),
                         "work": "mixed additions counted on the device per timed launch (sorted entries "
                                 "minus the pieces lanes start fresh, k_count_pieces) x 10 Fq products "
                                 "(8M+2S) / summed launch duration (HIP events on the library stream)",
                         "peak_basis": f"{mad_cycles():.2f} cycles per wave64 v_mad_u64_u32 per "
                                       f"SIMD (profiles/r02_ubench_ops.txt) x 1024 SIMDs x 2.4 GHz "
                                       f"/ {MADS_PER_FQ_PRODUCT} mads per Fq product",
                         "launches": acc_n,
                         "launch_ms": round(acc_avg_s * 1e3, 3),
                         "entries_per_launch": round(entries / max(acc_n, 1)),
                         "madds_per_launch": round(madds / max(acc_n, 1)),
                         "madds_per_proof": round(madds / args.steps),
                         "madds_per_s": round(madds_per_s / 1e9, 3),
                         "issue_model": {"peak_gmadd_s": round(valu_peak / 1e9, 3),
                                         "frac": round(madds_per_s / valu_peak, 4),
                                         "basis": "tools/isa_model.py: 19,761 SIMD cycles per 64 "
                                                  "mixed additions of the compiled kernel",
                                         "held_clock_ghz": HELD_CLOCK_GHZ,
                                         "frac_at_held_clock": round(held, 4),
                                         "exceeds_ceiling": held > 1.0,
                                         "held_clock_basis": "GRBM_GUI_ACTIVE / 8 XCDs / kernel time "
                                                             "(profiles/r02_pmc_clock.txt)"},
                         "dense_equivalent": {
                             "entries_per_launch": round(dense / max(acc_n, 1)),
                             "gmadd_s": round(dense / acc_s / 1e9, 3) if acc_s > 0 else 0.0,
                             "note": "MSMs x windows x points per launch: the work a dense Pippenger "
                                     "over the same MSMs does (zero digits, copy groups and padding "
                                     "rows drop out of the real count); not the kernel's work"},
                         "redo_lanes_per_proof": round(redo_lanes / args.steps, 2),
                         "exact_fallbacks_per_proof": round(exact_fallbacks / args.steps, 2),
                         "hbm": {"achieved_gbs": round(achieved, 1), "peak_gbs": HBM_PEAK_GBS,
                                 "frac": round(achieved / HBM_PEAK_GBS, 5),
                                 "algorithmic_bytes_per_launch": round(alg_per_launch),
                                 "basis": f"{ALG_BYTES_PER_ENTRY} B per sorted entry (one 96-B affine "
                                          "point + its 4-B index) x real entries",
                                 # SURVEY 8(d)'s per-MSM figure: every point and scalar once,
                                 # n (96 + 32) B; the folded table reads one 128-B line per
                                 # (point, window) instead, trading bytes for the doublings
                                 "survey_bytes_per_launch": round(dense / max(acc_n, 1) / msm_windows(args.lg) * 128),
                                 "traffic_over_survey": (round(traffic / (dense / max(acc_n, 1) / msm_windows(args.lg) * 128), 2)
                                                         if traffic and dense else None)},
                         "quotient": quotient_roofline(q_ms, q_n, q_gbs, q_points, q_prods,
                                                       args.circuit == "merkle")},
            "stages_ms": {k: round(v, 2) for k, v in stages},
            "hbm_gbs": round(proof_bytes / per_proof / 1e9, 1),
            "hbm_whole_proof": {"bytes_per_proof": round(proof_bytes), "achieved_gbs": round(proof_bytes / per_proof / 1e9, 1),
                                "peak_gbs": HBM_PEAK_GBS, "frac": round(proof_bytes / per_proof / 1e9 / HBM_PEAK_GBS, 4),
                                "basis": "this rank's algorithmic bytes per proof / the proof's wall-clock: "
                                         "prover op credits (prover.cpp alg(): transforms 2 x 32 B per element, "
                                         "LDEs (1 + blocks) x 32 B, quotient (inputs + 1) x 32 B per point, "
                                         "scans, combinations, gathers) + MSM scalars (32 B) + 100 B per sorted "
                                         "entry (DESIGN.md 5)",
                                "breakdown_gb": {"ops": round(ctx.kernel_bytes("proof_alg_bytes") / args.steps / 1e9, 2),
                                                 "msm_scalars": round(ctx.kernel_bytes("msm_scalar_bytes") / args.steps / 1e9, 2),
                                                 "msm_entries": round(entries * ALG_BYTES_PER_ENTRY / args.steps / 1e9, 2)}},
        }
        slots = {"slotted_batches_per_proof": round(slot_batches / args.steps, 2),
                 "slot_overflows_per_proof": round(slot_overflows / args.steps, 2),
                 # summed over the timed batches: the busiest range's records x world / all records
                 "bucket_range_balance": (round(dest_max * max(world, solo.world if solo else 1) / dest_sum, 4)
                                          if dest_sum else None)}
        if ex is not None:
            k = args.steps + args.warmup
            out["exchange"] = {"backend": ex.backend, "stream_ordered": ex.ordered, **slots,
                               "callbacks_per_proof": timed_cb["callbacks"],
                               "callback_ms_per_proof": round(timed_cb["callback_ms"], 3),
                               "callbacks_per_proof_incl_warmup": (ex.calls + ex.a2a_calls + getattr(ex, "v_calls", 0)) / k}
        if solo:
            # xGMI term the loopback leaves out: one
            # direct link per peer on a fully connected 8-GPU node, all peers
            # in parallel, so a collective costs its bytes per peer over one
            # link's rate plus a per-collective latency.  Stated assumptions
            # (PNP_XGMI_LINK_GBS, PNP_XGMI_LAT_US): 64 GB/s per link and
            # direction (MI355X quotes ~153 GB/s per link, both directions;
            # RCCL reaches ~80% of it), 25 us per collective
            link = float(os.environ.get("PNP_XGMI_LINK_GBS", "64")) * 1e9
            lat = float(os.environ.get("PNP_XGMI_LAT_US", "25")) * 1e-6
            k = args.steps + args.warmup
            peers = max(solo.world - 1, 1)
            per_peer = ((solo.a2a_bytes_moved + solo.v_bytes_moved) / k / peers
                        + solo.gather_bytes / k / solo.world)  # an all-gather slot goes to every peer
            xgmi_s = per_peer / link + timed_cb["callbacks"] * lat
            xgmi = {"ms_per_proof": round(xgmi_s * 1e3, 3),
                    "bytes_per_peer_per_proof": round(per_peer),
                    "collectives_per_proof": timed_cb["callbacks"],
                    "link_gbs_per_direction": link / 1e9, "latency_us_per_collective": lat * 1e6,
                    "projected_rank_ms": round(per_proof * 1e3 + xgmi_s * 1e3, 2),
                    "basis": "(all-to-all + bucket-record bytes sent / (world - 1) + all-gather slot bytes) "
                             "/ one link's rate + collectives x latency; not overlapped with compute "
                             "(an upper bound for the exchanges the proof waits on)"}
            out["solo"] = {"rank": solo.rank, "world": solo.world, "xgmi_model": xgmi,
                           "allgathers_per_proof": timed_cb["allgathers"],
                           "alltoalls_per_proof": timed_cb["alltoalls"],
                           "allgather_bytes_per_proof": solo.gather_bytes / (args.steps + args.warmup),
                           "alltoall_bytes_sent_per_proof": solo.a2a_bytes_moved / (args.steps + args.warmup),
                           "bucket_alltoallvs_per_proof": timed_cb["bucket_alltoallvs"],
                           "bucket_bytes_sent_per_proof": solo.v_bytes_moved / (args.steps + args.warmup),
                           "callbacks_per_proof": timed_cb["callbacks"],
                           # records this rank's points send to each bucket range: max / mean
                           # (1 = every range gets its share; the unscaled top window gave
                           # range 0 ~1.67x at 8 ranks), and the fixed-slot exchange's use
                           **slots,
                           "callback_ms_per_proof": round(timed_cb["callback_ms"], 3),
                           "ordered": solo.ordered,
                           # the (meaningless, deterministic) proof bytes: the same with the
                           # ordered and the synchronised loopback (tests/test_gpu_rccl.py)
                           "proof_sha256": __import__("hashlib").sha256(abi.proof_to_bytes(proof)).hexdigest(),
                           "note": "per-rank work of a W-GPU proof; the collectives are loopbacks "
                                   "(their xGMI time is not included; callback_ms is the host time "
                                   "spent inside the loopback callbacks — when ordered (enqueued on the "
                                   "library stream without host syncs, as the RCCL exchange) it includes "
                                   "the host waiting for queue space while it runs ahead of the GPU)"}
        if not args.no_verify:
            chk = check_proof(syn, proof, args.circuit)
            out["verified"] = chk.pop("verified") and all_equal
            out["verification"] = chk
            log(f"proof check: {out['verified']} {chk}")
        if args.drop_in and world == 1:
            out["drop_in"] = drop_in(ctx, syn, args.steps, v1=args.drop_in == "v1")
            if cold:
                out["drop_in"].update(cold)
        if args.cpu_lg and world == 1:  # the CPU baseline: rank 0 at N = 1 only
            try:
                out["cpu_baseline"] = cpu_baseline(ctx, args.cpu_lg, args.circuit, syn, proofs[0])
            except Exception as e:  # the CPU leg must never hide the GPU number
                out["cpu_baseline"] = {"error": repr(e)}
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()
    if rank == 0 and out.get("verified") is False:
        log("bench: the timed proof did NOT verify")
        return 3


if __name__ == "__main__":
    sys.exit(main() or 0)
