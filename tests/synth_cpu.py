"""CPU mirror of bench.py's Synthetic instance (the HEIGHT=15-shaped input the
bench proves), built with the oracle's generators (oracle/synth.c mirrors
csrc/synth.hip) so the CPU restatement can prove exactly the instance the
GPU proves.  Test infrastructure only.

    syn = SyntheticCPU(lg, gates, seed)    # same arrays as bench.Synthetic
    proof = syn.oracle_proof()
"""
import ctypes as C

import numpy as np

from pnp_testlib import oracle, vp, ptr_of, VK_POLYS, verifier_key  # noqa: I001 (sets sys.path)
from pnp import abi

POLYS = ("q_l", "q_r", "q_o", "q_4", "q_c", "q_hl", "q_hr", "q_h4", "q_arith",
         "left_sigma", "right_sigma", "out_sigma", "fourth_sigma")
SEL_IN = ("q_l", "q_r", "q_o", "q_4", "q_c", "q_hl", "q_hr", "q_h4")
PI_POS = 7


def _lib():
    lib = oracle()
    if not getattr(lib, "_synth_sig", False):
        v = C.c_void_p
        lib.or_synth_random_fr.argtypes = [v, C.c_uint64, C.c_uint64]
        lib.or_synth_circuit.argtypes = [C.c_void_p * 4, C.c_void_p * 9, C.c_void_p * 4, C.c_uint64,
                                         C.c_uint64, C.c_uint64, v]
        lib.or_synth_coset_consts.argtypes = [v, v, C.c_uint32]
        lib.or_synth_merkle.argtypes = [C.c_uint32, v, v, v, v, C.c_void_p * 4, C.c_void_p * 9,
                                        C.c_void_p * 4, C.c_uint64, v]
        lib.or_synth_merkle.restype = C.c_int
        lib._synth_sig = True
    return lib


def merkle_gates(height: int) -> int:
    return 193 * ((1 << (height - 1)) - 1) + 5


class SyntheticCPU:
    """bench.Synthetic(ctx, lg, gates, seed, circuit) rebuilt on the CPU.

    circuit="merkle": the reference's Poseidon Merkle circuit of HEIGHT
    lg - 7 (or_synth_merkle mirrors pnp_synth_merkle; `gates` is ignored),
    random leaves / blinding values from the same seeds as bench.py, PI =
    -root at the root row.  circuit="arith": the round-1 stand-in."""

    def __init__(self, lg_n: int, gates: int, seed: int, keep_evals: bool = True, circuit: str = "arith"):
        lib = _lib()
        n, N8 = 1 << lg_n, 8 << lg_n
        self.n, self.lg_n, self.seed, self.circuit_kind = n, lg_n, seed, circuit
        a = self.arrays = {}
        s = seed * 1000

        def rnd(cnt, sd):
            x = np.zeros((cnt, 4), dtype=np.uint64)
            lib.or_synth_random_fr(vp(x), cnt, sd)
            return x

        nev = {p: np.zeros((n, 4), dtype=np.uint64) for p in POLYS}
        if circuit == "merkle":
            from poseidon import PoseidonConstants, flat_constants
            from pnp_testlib import fr_mont, ints_to_arr, R_MOD
            height = self.height = lg_n - 7
            gates = merkle_gates(height)
            for k in ("w_l", "w_r", "w_o", "w_4"):
                a[k] = np.zeros((gates, 4), dtype=np.uint64)
            leaves, blind = rnd(1 << (height - 1), s + 1), rnd(8, s + 2)
            self.nodes = np.zeros(((1 << (height - 1)) - 1, 4), dtype=np.uint64)
            pc = ints_to_arr([fr_mont(v) for v in flat_constants(PoseidonConstants())])
            W = (C.c_void_p * 4)(*[a[k].ctypes.data for k in ("w_l", "w_r", "w_o", "w_4")])
            S = (C.c_void_p * 9)(*[nev[k].ctypes.data for k in SEL_IN + ("q_arith",)])
            G = (C.c_void_p * 4)(*[nev[k].ctypes.data for k in ("left_sigma", "right_sigma", "out_sigma",
                                                                 "fourth_sigma")])
            root = np.zeros(4, dtype=np.uint64)
            rc = lib.or_synth_merkle(height, vp(pc), vp(leaves), vp(blind), vp(self.nodes), W, S, G, n,
                                     vp(root))
            assert rc == 0, rc
            self.root = sum(int(root[k]) << (64 * k) for k in range(4))
            neg = (-self.root) % R_MOD
            self.pi_canon = [(neg >> (64 * k)) & (2**64 - 1) for k in range(4)]
            self.pi_pos = gates - 1
        else:
            a["w_l"] = rnd(gates, s + 1)
            a["w_4"] = rnd(gates, s + 4)
            a["w_r"] = np.zeros((gates, 4), dtype=np.uint64)
            a["w_o"] = np.zeros((gates, 4), dtype=np.uint64)
            self.pi_canon = [123456789 + seed, 0, 0, 0]
            self.pi_pos = PI_POS
            for i, p in enumerate(SEL_IN):
                nev[p] = rnd(n, s + 100 + i)
            W = (C.c_void_p * 4)(*[a[k].ctypes.data for k in ("w_l", "w_r", "w_o", "w_4")])
            S = (C.c_void_p * 9)(*[nev[k].ctypes.data for k in SEL_IN + ("q_arith",)])
            G = (C.c_void_p * 4)(*[nev[k].ctypes.data for k in ("left_sigma", "right_sigma", "out_sigma",
                                                                 "fourth_sigma")])
            pi = np.array(self.pi_canon, dtype=np.uint64)
            lib.or_synth_circuit(W, S, G, n, gates, PI_POS, vp(pi))
        self.gates = gates
        a["q_lookup"] = np.zeros((gates, 4), dtype=np.uint64)
        a["pi"] = np.array(self.pi_canon, dtype=np.uint64)
        self.nevals = {p: nev[p].copy() for p in POLYS} if lg_n <= 16 else None
        for p in POLYS:
            c = nev.pop(p)
            lib.or_ntt(vp(c), lg_n, 1, 0)  # coefficients of the n-domain evaluations
            a[p + "_coeffs"] = c
            if keep_evals:
                e = np.zeros((N8, 4), dtype=np.uint64)
                lib.or_coset_lde8(vp(c), vp(e), lg_n)
                a[p + "_evals"] = e
        if keep_evals:
            a["zero8"] = np.zeros((N8, 4), dtype=np.uint64)
            a["linear_evaluations"] = np.zeros((N8, 4), dtype=np.uint64)
            a["v_h_coset_8n"] = np.zeros((N8, 4), dtype=np.uint64)
            lib.or_synth_coset_consts(vp(a["v_h_coset_8n"]), vp(a["linear_evaluations"]), lg_n)
        a["zero_n"] = np.zeros((n, 4), dtype=np.uint64)
        a["empty"] = np.zeros((1, 4), dtype=np.uint64)
        self.tau_mont = rnd(1, s + 999)
        a["srs"] = np.zeros((n, 12), dtype=np.uint64)
        lib.or_srs(vp(a["srs"]), n, vp(self.tau_mont))
        a["gamma_g"] = np.zeros((2, 12), dtype=np.uint64)
        self._structs(keep_evals)

    def _structs(self, keep_evals):
        a = self.arrays
        self.circuit = abi.CircuitC(n=self.gates, lookup_len=0, intended_pi_pos=self.pi_pos,
                                    q_lookup=ptr_of(a["q_lookup"]), pi=ptr_of(a["pi"]),
                                    w_l=ptr_of(a["w_l"]), w_r=ptr_of(a["w_r"]), w_o=ptr_of(a["w_o"]),
                                    w_4=ptr_of(a["w_4"]))
        pk = abi.ProverKeyC()
        for f in abi.PK_FIELDS:
            if f in a:
                key = f
            elif f.endswith("_evals"):
                key = "zero8" if keep_evals else "empty"
            elif f.startswith("table"):
                key = "zero_n"
            else:
                key = "empty"  # q_m / custom-selector / q_lookup coeffs: empty Rust Vecs
            setattr(pk, f, ptr_of(a[key]))
        self.pk = pk
        self.ck = abi.CommitKeyC(powers_of_g=ptr_of(a["srs"]), powers_of_gamma_g=ptr_of(a["gamma_g"]))

    def oracle_proof(self) -> abi.ProofC:
        out = abi.ProofC()
        rc = oracle().or_gen_proof(C.byref(self.circuit), C.byref(self.pk), C.byref(self.ck),
                                   C.byref(out))
        assert rc == 0, rc
        return out

    def vk(self) -> np.ndarray:
        a = self.arrays
        return verifier_key({k: a[k + "_coeffs"] for k in VK_POLYS if k + "_coeffs" in a}, self.n,
                            a["srs"])

    def pis(self):
        return [(self.pi_pos, sum(int(v) << (64 * k) for k, v in enumerate(self.pi_canon)))]
