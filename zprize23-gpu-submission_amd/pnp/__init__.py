"""Python host mirror of the gen_proof C-ABI (include/pnp_plonk.h).

The reference host is Rust: Prover::prove_pnp (plonk-core/src/proof_system/
prover.rs:693-907) marshals CircuitC / ProverKeyC / CommitKeyC and calls the
extern "C" gen_proof (plonk-core/src/lib.rs:237-239).  Rust is not available
in this image, so tests and the bench drive the same ABI through ctypes:

    lib = pnp.load()                      # libpnp_plonk.so, fails loudly if absent
    proof = lib.gen_proof(circuit, pk, ck)   # v1, by value, like lib.rs

plus the v2 resident-key API (Context) used by the bench.  This package holds
no compute: every field/curve operation runs in the HIP library.
"""
import ctypes as C
import os

from . import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PNP_PLONK_LIB",
                          os.path.join(os.path.dirname(_HERE), "lib", "libpnp_plonk.so"))
_LIB = None

PNP_OK = 0
ERRORS = {-1: "PNP_E_ARG", -2: "PNP_E_DEVICE", -3: "PNP_E_NOKEY", -4: "PNP_E_ENVELOPE",
          -5: "PNP_E_NOMEM"}

# exported symbols declared by include/pnp_plonk.h (checked by tests/test_abi.py)
SYMBOLS = ("gen_proof", "pnp_last_error", "pnp_ctx_create", "pnp_ctx_destroy",
           "pnp_load_prover_key", "pnp_load_commit_key", "pnp_prove", "pnp_prove_ex",
           "pnp_last_stage_times",
           "pnp_kernel_timing", "pnp_kernel_stats", "pnp_kernel_bytes", "pnp_set_msm_shard",
           "pnp_set_exchange_a2a",
           "pnp_sync", "pnp_ntt", "pnp_coset_lde8", "pnp_commit", "pnp_commit_ck", "pnp_commit_evals", "pnp_poly_eval",
           "pnp_poly_div_linear", "pnp_prefix_product", "pnp_batch_inverse",
           "pnp_synth_random_fr", "pnp_synth_srs", "pnp_synth_coset_consts", "pnp_synth_circuit",
           "pnp_synth_merkle", "pnp_load_commit_key_strided", "pnp_proof_infinity_mask",
           "pnp_set_exchange_v", "pnp_commit_segments", "pnp_hbm_usage",
           "pnp_ctx_stream", "pnp_set_exchange_ordered", "pnp_v1_context")


# int allgather(void *user, uint64_t bytes_per_rank) — pnp_set_msm_shard
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_uint64)
# int alltoall(void *user, uint64_t bytes_per_peer) — pnp_set_exchange_a2a
ALLTOALL_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_uint64)
# int alltoallv(void *user, const uint64_t *send_bytes, const uint64_t *recv_bytes) — pnp_set_exchange_v
ALLTOALLV_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64))


class PnpError(RuntimeError):
    pass


def load(path: str = LIB_PATH):
    """Load the HIP library.  There is no CPU fallback: a missing library raises."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise PnpError(f"{path} not built (run __graft_entry__.build() or make -C csrc)")
    # One HIP runtime per process: torch bundles its own libamdhip64.so.7.  If
    # our library were loaded first it would pull /opt/rocm's copy and torch's
    # later HSA init fails ("No HIP GPUs are available").  Loading torch first
    # makes the soname resolve to the already-loaded runtime for both.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    vp, u64, i32 = C.c_void_p, C.c_uint64, C.c_int
    lib.gen_proof.argtypes = [abi.CircuitC, abi.ProverKeyC, abi.CommitKeyC]
    lib.gen_proof.restype = abi.ProofC
    lib.pnp_v1_context.restype = vp
    lib.pnp_last_error.restype = C.c_char_p
    lib.pnp_ctx_create.argtypes = [i32, C.POINTER(vp)]
    lib.pnp_ctx_destroy.argtypes = [vp]
    lib.pnp_ctx_destroy.restype = None
    lib.pnp_load_prover_key.argtypes = [vp, C.POINTER(abi.ProverKeyC), u64, i32]
    lib.pnp_load_commit_key.argtypes = [vp, C.POINTER(abi.CommitKeyC), u64, i32]
    lib.pnp_prove.argtypes = [vp, C.POINTER(abi.CircuitC), i32, C.POINTER(abi.ProofC)]
    lib.pnp_prove_ex.argtypes = [vp, C.POINTER(abi.CircuitC), i32, u64, vp, vp, C.c_char_p,
                                 C.POINTER(abi.ProofC)]
    lib.pnp_last_stage_times.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_char_p), i32]
    lib.pnp_kernel_timing.argtypes = [vp, i32]
    lib.pnp_kernel_stats.argtypes = [vp, C.c_char_p, C.POINTER(C.c_double), C.POINTER(C.c_int)]
    lib.pnp_kernel_bytes.argtypes = [vp, C.c_char_p, C.POINTER(C.c_double)]
    lib.pnp_set_msm_shard.argtypes = [vp, i32, i32, ALLGATHER_FN, vp, vp, u64]
    lib.pnp_set_exchange_a2a.argtypes = [vp, ALLTOALL_FN, vp, vp, u64]
    lib.pnp_set_exchange_v.argtypes = [vp, ALLTOALLV_FN, vp, vp, vp, u64]
    lib.pnp_sync.argtypes = [vp]
    lib.pnp_ntt.argtypes = [vp, vp, C.c_uint32, i32, i32]
    lib.pnp_coset_lde8.argtypes = [vp, vp, vp, C.c_uint32]
    lib.pnp_commit.argtypes = [vp, vp, vp, u64, C.POINTER(abi.CommitmentC)]
    lib.pnp_commit_ck.argtypes = [vp, vp, u64, C.POINTER(abi.CommitmentC)]
    lib.pnp_commit_evals.argtypes = [vp, vp, u64, C.POINTER(abi.CommitmentC)]
    lib.pnp_hbm_usage.argtypes = [vp, C.POINTER(u64)]
    lib.pnp_ctx_stream.argtypes = [vp, C.POINTER(vp)]
    lib.pnp_set_exchange_ordered.argtypes = [vp, i32]
    lib.pnp_commit_segments.argtypes = [vp, vp, u64, i32, C.POINTER(u64), C.POINTER(vp), u64,
                                        C.POINTER(abi.CommitmentC)]
    lib.pnp_poly_eval.argtypes = [vp, vp, u64, vp, vp]
    lib.pnp_poly_div_linear.argtypes = [vp, vp, u64, vp]
    lib.pnp_prefix_product.argtypes = [vp, vp, u64]
    lib.pnp_batch_inverse.argtypes = [vp, vp, u64]
    lib.pnp_synth_random_fr.argtypes = [vp, vp, u64, u64]
    lib.pnp_synth_srs.argtypes = [vp, vp, u64, vp]
    lib.pnp_synth_coset_consts.argtypes = [vp, vp, vp, C.c_uint32]
    lib.pnp_synth_circuit.argtypes = [vp, C.c_void_p * 4, C.c_void_p * 9, C.c_void_p * 4, u64, u64,
                                      u64, vp]
    lib.pnp_synth_merkle.argtypes = [vp, C.c_uint32, vp, vp, vp, vp, C.c_void_p * 4, C.c_void_p * 9,
                                     C.c_void_p * 4, u64, vp]
    lib.pnp_load_commit_key_strided.argtypes = [vp, vp, u64, C.POINTER(abi.AffineLayout), i32]
    lib.pnp_proof_infinity_mask.argtypes = [C.POINTER(abi.ProofC)]
    for name in SYMBOLS:
        if name.startswith("pnp_") and name not in ("pnp_last_error", "pnp_ctx_destroy", "pnp_v1_context"):
            getattr(lib, name).restype = C.c_int if name != "pnp_last_error" else C.c_char_p
    lib.pnp_proof_infinity_mask.restype = C.c_uint32
    _LIB = lib
    return lib


def infinity_mask(proof: abi.ProofC) -> int:
    """pnp_proof_infinity_mask: bit k set when the k-th commitment of the
    ProofC (abi.PROOF_COMMITMENTS order) is the point at infinity."""
    return int(load().pnp_proof_infinity_mask(C.byref(proof)))


def infinity_flags(proof: abi.ProofC) -> dict:
    m = infinity_mask(proof)
    return {name: bool((m >> k) & 1) for k, name in enumerate(abi.PROOF_COMMITMENTS)}


def check(rc: int, what: str = ""):
    if rc != PNP_OK:
        msg = load().pnp_last_error()
        raise PnpError(f"{what}: {ERRORS.get(rc, rc)}: {msg.decode() if msg else ''}")


class Context:
    """One MI355X: stream, NTT tables, MSM buffers and HBM-resident keys."""

    def __init__(self, device: int = 0):
        self.lib = load()
        h = C.c_void_p()
        check(self.lib.pnp_ctx_create(device, C.byref(h)), "pnp_ctx_create")
        self.h = h

    def close(self):
        if self.h:
            self.lib.pnp_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- keys / prove
    def load_prover_key(self, pk: abi.ProverKeyC, domain: int, device_ptrs: bool):
        check(self.lib.pnp_load_prover_key(self.h, C.byref(pk), domain, int(device_ptrs)),
              "pnp_load_prover_key")

    def load_commit_key(self, ck: abi.CommitKeyC, n_points: int, device_ptrs: bool):
        check(self.lib.pnp_load_commit_key(self.h, C.byref(ck), n_points, int(device_ptrs)),
              "pnp_load_commit_key")

    def load_commit_key_strided(self, points: int, n_points: int, layout: abi.AffineLayout = abi.ARK_G1_AFFINE,
                                device_ptrs: bool = False):
        """The SRS in arkworks' own G1Affine memory layout (prover.rs:700-711
        without the per-call conversion)."""
        check(self.lib.pnp_load_commit_key_strided(self.h, C.c_void_p(points), n_points, C.byref(layout),
                                                   int(device_ptrs)), "pnp_load_commit_key_strided")

    def prove(self, cs: abi.CircuitC, device_ptrs: bool) -> abi.ProofC:
        out = abi.ProofC()
        check(self.lib.pnp_prove(self.h, C.byref(cs), int(device_ptrs), C.byref(out)), "pnp_prove")
        return out

    def prove_ex(self, cs: abi.CircuitC, device_ptrs: bool, pis, label: bytes = b"Merkle tree"):
        """pnp_prove_ex: pis = [(position, canonical value int)], any order."""
        k = len(pis)
        pos = (C.c_uint64 * max(k, 1))(*[p for p, _ in pis])
        vals = (C.c_uint64 * max(4 * k, 1))()
        for i, (_, v) in enumerate(pis):
            for j in range(4):
                vals[4 * i + j] = (v >> (64 * j)) & 0xFFFFFFFFFFFFFFFF
        out = abi.ProofC()
        check(self.lib.pnp_prove_ex(self.h, C.byref(cs), int(device_ptrs), k, pos, vals, label,
                                    C.byref(out)), "pnp_prove_ex")
        return out

    def stage_times(self):
        cap = 64
        ms = (C.c_double * cap)()
        names = (C.c_char_p * cap)()
        k = self.lib.pnp_last_stage_times(self.h, ms, names, cap)
        return [(names[i].decode(), ms[i]) for i in range(min(k, cap))]

    def kernel_timing(self, enable: bool):
        check(self.lib.pnp_kernel_timing(self.h, int(enable)), "pnp_kernel_timing")

    def kernel_bytes(self, name: str) -> float:
        b = C.c_double()
        check(self.lib.pnp_kernel_bytes(self.h, name.encode(), C.byref(b)), "pnp_kernel_bytes")
        return b.value

    def set_msm_shard(self, exchange):
        """Window-sharded MSM across ranks (pnp_set_msm_shard); `exchange` is a
        pnp.shard.WindowExchange, or None to go back to single-GPU MSMs."""
        if exchange is None or exchange.world == 1:
            check(self.lib.pnp_set_exchange_ordered(self.h, 0), "pnp_set_exchange_ordered")
            check(self.lib.pnp_set_msm_shard(self.h, 0, 1, ALLGATHER_FN(), None, None, 0),
                  "pnp_set_msm_shard")
            check(self.lib.pnp_set_exchange_v(self.h, ALLTOALLV_FN(), None, None, None, 0), "pnp_set_exchange_v")
            self._exchange = None
            return
        # RCCL exchanges run on the library's stream, without host syncs
        import torch
        sp = C.c_void_p()
        check(self.lib.pnp_ctx_stream(self.h, C.byref(sp)), "pnp_ctx_stream")
        if exchange.buf.is_cuda and sp.value:
            exchange.stream = torch.cuda.ExternalStream(sp.value, device=exchange.buf.device)
        check(self.lib.pnp_set_exchange_ordered(self.h, int(exchange.ordered)), "pnp_set_exchange_ordered")
        cb = exchange.c_callback()
        check(self.lib.pnp_set_msm_shard(self.h, exchange.rank, exchange.world, cb, None,
                                         exchange.buf.data_ptr(), exchange.buf.numel() * 8),
              "pnp_set_msm_shard")
        keep = [exchange, cb]
        if exchange.a2a is not None:  # distributed round 4 (call before load_prover_key)
            cb2 = exchange.c_alltoall()
            check(self.lib.pnp_set_exchange_a2a(self.h, cb2, None, exchange.a2a.data_ptr(),
                                                exchange.a2a.numel() * 8), "pnp_set_exchange_a2a")
            keep.append(cb2)
        if getattr(exchange, "vsend", None) is not None:  # bucket-range MSMs
            cb3 = exchange.c_alltoallv()
            check(self.lib.pnp_set_exchange_v(self.h, cb3, None, exchange.vsend.data_ptr(),
                                              exchange.vrecv.data_ptr(), exchange.vsend.numel() * 8),
                  "pnp_set_exchange_v")
            keep.append(cb3)
        self._exchange = keep  # keep the callbacks alive

    def hbm_usage(self) -> dict:
        """pnp_hbm_usage: bytes held / peak, and the key-load plan's parts."""
        o = (C.c_uint64 * 6)()
        check(self.lib.pnp_hbm_usage(self.h, o), "pnp_hbm_usage")
        return dict(zip(("live", "peak", "mandatory", "lagrange", "groups", "transient"), list(o)))

    def kernel_stats(self, name: str):
        ms, cnt = C.c_double(), C.c_int()
        check(self.lib.pnp_kernel_stats(self.h, name.encode(), C.byref(ms), C.byref(cnt)),
              "pnp_kernel_stats")
        return ms.value, cnt.value

    # ---- operator API (HBM addresses as ints)
    def sync(self):
        check(self.lib.pnp_sync(self.h), "pnp_sync")

    def ntt(self, addr: int, lg_n: int, inverse: bool = False, coset: bool = False):
        check(self.lib.pnp_ntt(self.h, C.c_void_p(addr), lg_n, int(inverse), int(coset)), "pnp_ntt")

    def coset_lde8(self, src: int, dst: int, lg_n: int):
        check(self.lib.pnp_coset_lde8(self.h, C.c_void_p(src), C.c_void_p(dst), lg_n), "pnp_coset_lde8")

    def commit(self, points: int, scalars: int, n: int) -> abi.CommitmentC:
        out = abi.CommitmentC()
        check(self.lib.pnp_commit(self.h, C.c_void_p(points), C.c_void_p(scalars), n, C.byref(out)),
              "pnp_commit")
        return out

    def commit_ck(self, scalars: int, n: int) -> abi.CommitmentC:
        """Commitment against the resident commit key (folded fixed-base MSM)."""
        out = abi.CommitmentC()
        check(self.lib.pnp_commit_ck(self.h, C.c_void_p(scalars), n, C.byref(out)), "pnp_commit_ck")
        return out

    def commit_evals(self, evals: int, n: int) -> abi.CommitmentC:
        """Commitment of the polynomial with these n evaluations on the order-n
        subgroup, against the resident key in the Lagrange basis."""
        out = abi.CommitmentC()
        check(self.lib.pnp_commit_evals(self.h, C.c_void_p(evals), n, C.byref(out)), "pnp_commit_evals")
        return out

    def commit_segments(self, points: int, n_points: int, seg_off, scalars, n: int):
        """B MSMs over sub-ranges [seg_off[b], seg_off[b] + n) of one base set
        (pnp_commit_segments: one folded table over all n_points)."""
        B = len(seg_off)
        offs = (C.c_uint64 * B)(*seg_off)
        sc = (C.c_void_p * B)(*scalars)
        out = (abi.CommitmentC * B)()
        check(self.lib.pnp_commit_segments(self.h, C.c_void_p(points), n_points, B, offs, sc, n, out),
              "pnp_commit_segments")
        return list(out)

    def poly_eval(self, addr: int, n: int, x_limbs):
        x = (C.c_uint64 * 4)(*x_limbs)
        out = (C.c_uint64 * 4)()
        check(self.lib.pnp_poly_eval(self.h, C.c_void_p(addr), n, x, out), "pnp_poly_eval")
        return list(out)

    def poly_div_linear(self, addr: int, n: int, z_limbs):
        z = (C.c_uint64 * 4)(*z_limbs)
        check(self.lib.pnp_poly_div_linear(self.h, C.c_void_p(addr), n, z), "pnp_poly_div_linear")

    def prefix_product(self, addr: int, n: int):
        check(self.lib.pnp_prefix_product(self.h, C.c_void_p(addr), n), "pnp_prefix_product")

    def batch_inverse(self, addr: int, n: int):
        check(self.lib.pnp_batch_inverse(self.h, C.c_void_p(addr), n), "pnp_batch_inverse")

    def random_fr(self, addr: int, n: int, seed: int):
        check(self.lib.pnp_synth_random_fr(self.h, C.c_void_p(addr), n, seed), "pnp_synth_random_fr")

    def srs(self, addr: int, n: int, tau_limbs):
        t = (C.c_uint64 * 4)(*tau_limbs)
        check(self.lib.pnp_synth_srs(self.h, C.c_void_p(addr), n, t), "pnp_synth_srs")

    def synth_circuit(self, w, sel, sigma, n: int, n_gates: int, pi_pos: int, pi_limbs):
        """w: 4 addrs (a in, b out, c out, d in); sel: 9 addrs (8 in, q_arith out);
        sigma: 4 addrs out (see include/pnp_plonk.h)."""
        W = (C.c_void_p * 4)(*w)
        S = (C.c_void_p * 9)(*sel)
        G = (C.c_void_p * 4)(*sigma)
        p = (C.c_uint64 * 4)(*pi_limbs)
        check(self.lib.pnp_synth_circuit(self.h, W, S, G, n, n_gates, pi_pos, p), "pnp_synth_circuit")

    def synth_merkle(self, height: int, consts, leaves: int, blind: int, nodes: int, w, sel, sigma, n: int):
        """The reference's Poseidon Merkle circuit (include/pnp_plonk.h):
        consts = 199 canonical ints (round constants, MDS row-major, tag);
        leaves / blind / nodes / w / sel / sigma device addresses; returns the
        root (canonical int)."""
        cs = (C.c_uint64 * (4 * 199))(*[(v >> (64 * k)) & (2**64 - 1) for v in consts for k in range(4)])
        root = (C.c_uint64 * 4)()
        check(self.lib.pnp_synth_merkle(self.h, height, cs, C.c_void_p(leaves), C.c_void_p(blind),
                                        C.c_void_p(nodes), (C.c_void_p * 4)(*w), (C.c_void_p * 9)(*sel),
                                        (C.c_void_p * 4)(*sigma), n, root), "pnp_synth_merkle")
        return sum(int(root[k]) << (64 * k) for k in range(4))

    def coset_consts(self, vh: int, x: int, lg_n: int):
        check(self.lib.pnp_synth_coset_consts(self.h, C.c_void_p(vh), C.c_void_p(x), lg_n),
              "pnp_synth_coset_consts")
