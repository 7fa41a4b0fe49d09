"""Shared helpers for the parity tests: field constants, limb packing, the
oracle loader (oracle/liboracle.so, test infrastructure) and a seeded
synthetic-input builder for the gen_proof ABI structs.

Synthetic inputs mirror the Merkle-circuit prover key's structure
(SURVEY.md §8a parity envelope): random witness wires, arithmetic selectors
and sigma polynomials (8n coset evaluations = coset LDE of the coefficients),
q_m / custom-gate selectors / q_lookup / lookup tables all zero, one public
input, real coset points and Z_H values on the 8n coset, SRS = [tau^i] G.
"""
import ctypes as C
import os
import subprocess
import sys
import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "zprize23-gpu-submission_amd")
if PKG not in sys.path:
    sys.path.insert(0, PKG)

from pnp import abi  # noqa: E402

R_MOD = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
Q_MOD = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
R_FR = pow(2, 256, R_MOD)
R_FQ = pow(2, 384, Q_MOD)
FR_ROOT32_MONT = [13381757501831005802, 6564924994866501612, 789602057691799140, 6625830629041353339]
FR_GEN = 7


def to_limbs(x: int, nlimbs: int):
    return [(x >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(nlimbs)]


def from_limbs(limbs) -> int:
    return sum(int(v) << (64 * i) for i, v in enumerate(limbs))


def fr_mont(x: int) -> int:
    return x * R_FR % R_MOD


def fr_unmont(x: int) -> int:
    return x * pow(R_FR, -1, R_MOD) % R_MOD


def fq_mont(x: int) -> int:
    return x * R_FQ % Q_MOD


def fq_unmont(x: int) -> int:
    return x * pow(R_FQ, -1, Q_MOD) % Q_MOD


def fr_root(lg: int) -> int:
    """canonical primitive 2^lg-th root of unity (domain.cu:29-36)"""
    w = fr_unmont(from_limbs(FR_ROOT32_MONT))
    return pow(w, 1 << (32 - lg), R_MOD)


def ints_to_arr(vals, nlimbs=4) -> np.ndarray:
    out = np.zeros((len(vals), nlimbs), dtype=np.uint64)
    for i, v in enumerate(vals):
        out[i] = to_limbs(int(v), nlimbs)
    return out


def arr_to_ints(arr) -> list:
    a = np.asarray(arr, dtype=np.uint64).reshape(-1, arr.shape[-1] if arr.ndim > 1 else 4)
    return [from_limbs(row) for row in a]


def rand_fr_mont_arr(rng: np.random.Generator, n: int) -> np.ndarray:
    """n Montgomery-form Fr values (uniform canonical values, then x*R mod r)."""
    raw = rng.integers(0, 2**64, size=(n, 4), dtype=np.uint64)
    raw[:, 3] &= np.uint64(0x7FFFFFFFFFFFFFFF)
    vals = [from_limbs(r) % R_MOD for r in raw]
    return ints_to_arr([fr_mont(v) for v in vals])


def ptr_of(a: np.ndarray):
    return a.ctypes.data_as(abi.U64P)


# ------------------------------------------------------------------ oracle
_ORACLE = None


def build_oracle():
    d = os.path.join(REPO, "oracle")
    subprocess.run(["make", "-s", "-C", d, "liboracle.so"], check=True)


def oracle():
    """oracle/liboracle.so (built on demand).  Test infrastructure only."""
    global _ORACLE
    if _ORACLE is None:
        build_oracle()
        lib = C.CDLL(os.path.join(REPO, "oracle", "liboracle.so"))
        vp = C.c_void_p
        lib.or_ntt.argtypes = [vp, C.c_uint32, C.c_int, C.c_int]
        lib.or_coset_lde8.argtypes = [vp, vp, C.c_uint32]
        lib.or_poly_eval.argtypes = [vp, C.c_uint64, vp, vp]
        lib.or_poly_div_linear.argtypes = [vp, C.c_uint64, vp]
        lib.or_prefix_product.argtypes = [vp, C.c_uint64]
        lib.or_batch_inverse.argtypes = [vp, C.c_uint64]
        lib.or_srs.argtypes = [vp, C.c_uint64, vp]
        lib.or_commit.argtypes = [vp, vp, C.c_uint64, vp]
        lib.or_fr_vec_to_mont.argtypes = [vp, C.c_uint64]
        lib.or_fr_vec_from_mont.argtypes = [vp, C.c_uint64]
        lib.or_transcript_new.restype = vp
        lib.or_transcript_new.argtypes = [C.c_char_p]
        lib.or_transcript_free.argtypes = [vp]
        lib.or_transcript_append_message.argtypes = [vp, C.c_char_p, vp, C.c_size_t]
        lib.or_transcript_append_scalar.argtypes = [vp, C.c_char_p, vp]
        lib.or_transcript_append_point.argtypes = [vp, C.c_char_p, vp]
        lib.or_transcript_append_pi.argtypes = [vp, C.c_char_p, vp, C.c_uint64]
        lib.or_transcript_challenge_bytes.argtypes = [vp, C.c_char_p, vp, C.c_size_t]
        lib.or_transcript_challenge_scalar.argtypes = [vp, C.c_char_p, vp]
        lib.or_gen_proof.argtypes = [vp, vp, vp, vp]
        lib.or_gen_proof.restype = C.c_int
        lib.or_num_threads.restype = C.c_int
        lib.or_set_num_threads.argtypes = [C.c_int]
        _ORACLE = lib
    return _ORACLE


def vp(a: np.ndarray):
    """Pointer to a's data that keeps a alive for as long as the pointer
    (vp(x.copy()) would otherwise hand C a freed temporary)."""
    p = C.c_void_p(a.ctypes.data)
    p._keep = a
    return p


# ------------------------------------------------------------------ synthetic inputs
PK_ZERO_EVALS = ("q_m_evals", "range_selector_evals", "logic_selector_evals",
                 "fixed_group_add_selector_evals", "variable_group_add_selector_evals",
                 "q_lookup_evals")
PK_RANDOM_COEFFS = ("q_l", "q_r", "q_o", "q_4", "q_c", "q_hl", "q_hr", "q_h4", "q_arith",
                    "left_sigma", "right_sigma", "out_sigma", "fourth_sigma")


def perm_mult(n_gates: int) -> int:
    """Multiplier A of the row permutation pi(i) = (A*i + 1) mod n_gates."""
    import math
    A = 0x9E3779B1 % n_gates if n_gates > 2 else 1
    while math.gcd(A, n_gates) != 1:
        A += 1
    return A


def satisfying_witness(sel, a, d, n_gates, pi_pos, pi_mont, lg_n):
    """Solve a satisfying witness / sigma for random arithmetic gates.

    Gate row i (q_arith = 1 for i < n_gates, 0 on padding rows):
        q_l a + q_r b + q_o c + q_4 d + q_hl a^5 + q_hr b^5 + q_h4 d^5 + q_c (+ PI_i) = 0
    Copy constraints: b_i = a_pi(i), pi(i) = (A i + 1) mod n_gates, giving the
    2-cycles {(b, i), (a, pi(i))}; c and d slots map to themselves.
    All values are canonical ints; returns (b, c, sigma[4]) canonical ints.
    Mirrored on the GPU by pnp_synth_circuit (csrc/synth.hip)."""
    n = 1 << lg_n
    w = fr_root(lg_n)
    A = perm_mult(n_gates)
    K = [1, 7, 13, 17]
    b = [0] * n
    c = [0] * n
    sig = [[0] * n for _ in range(4)]
    wp = [pow(w, i, R_MOD) for i in range(n)]
    for i in range(n):
        for j in range(4):
            sig[j][i] = K[j] * wp[i] % R_MOD
    for i in range(n_gates):
        pi_i = (A * i + 1) % n_gates
        b[i] = a[pi_i]
        sig[1][i] = wp[pi_i]                      # (b, i) -> (a, pi(i))
        sig[0][pi_i] = 7 * wp[i] % R_MOD          # (a, pi(i)) -> (b, i)
        ql, qr, qo, q4, qc, qhl, qhr, qh4 = (sel[k][i] for k in
                                             ("q_l", "q_r", "q_o", "q_4", "q_c", "q_hl", "q_hr", "q_h4"))
        acc = (ql * a[i] + qr * b[i] + q4 * d[i] + qhl * pow(a[i], 5, R_MOD) + qhr * pow(b[i], 5, R_MOD)
               + qh4 * pow(d[i], 5, R_MOD) + qc) % R_MOD
        if i == pi_pos:
            acc = (acc + fr_unmont(pi_mont)) % R_MOD
        c[i] = (-acc) * pow(qo, -1, R_MOD) % R_MOD
    return b, c, sig


class Inputs:
    """Host-resident synthetic gen_proof inputs + the ctypes structs over them.

    satisfying=True (default): a satisfying random arithmetic circuit with copy
    constraints (see satisfying_witness), so the quotient has degree < 6n and
    t_7 = t_8 = 0 exactly as in the real Merkle circuit.  satisfying=False:
    independent random witness / selectors / sigmas (still valid inputs).
    lookup_rows > 0: that many random gates get a non-zero q_lookup witness, so
    the query table f is non-zero and z2 is a real grand product (the general
    lookup branch); qm_qlookup_evals: random q_m / q_lookup 8n evaluations, so
    the quotient's q_m and q_lookup terms are live."""

    def __init__(self, lg_n: int, seed: int, n_gates: int | None = None, pi_pos: int = 3,
                 satisfying: bool = True, lookup_rows: int = 0, qm_qlookup_evals: bool = False):
        lib = oracle()
        rng = np.random.default_rng(seed)
        n = 1 << lg_n
        N8 = 8 * n
        self.lg_n, self.n = lg_n, n
        self.n_gates = n_gates if n_gates is not None else n - 3
        self.pi_pos = pi_pos
        self.arrays = {}
        a = self.arrays
        ng = self.n_gates
        a["pi"] = np.array(to_limbs(int(rng.integers(1, 2**62)), 4), dtype=np.uint64)
        a["q_lookup"] = np.zeros((ng, 4), dtype=np.uint64)

        def rnd(cnt):
            return [int(v) for v in (from_limbs(r) % R_MOD for r in
                                     rng.integers(0, 2**64, size=(cnt, 4), dtype=np.uint64))]

        def mont_arr(vals):
            return ints_to_arr([fr_mont(v) for v in vals])

        evals = {}
        if satisfying:
            sel = {k: rnd(ng) + [0] * (n - ng) for k in
                   ("q_l", "q_r", "q_o", "q_4", "q_c", "q_hl", "q_hr", "q_h4")}
            sel["q_arith"] = [1] * ng + [0] * (n - ng)
            wa, wd = rnd(ng) + [0] * (n - ng), rnd(ng) + [0] * (n - ng)
            pi_m = fr_mont(from_limbs(a["pi"]) % R_MOD)
            wb, wc, sig = satisfying_witness(sel, wa, wd, ng, pi_pos, pi_m, lg_n)
            for k, v in sel.items():
                evals[k] = v
            for j, name in enumerate(("left_sigma", "right_sigma", "out_sigma", "fourth_sigma")):
                evals[name] = sig[j]
            for name, vals in (("w_l", wa), ("w_r", wb), ("w_o", wc), ("w_4", wd)):
                a[name] = mont_arr(vals[:ng])
        else:
            for name in ("w_l", "w_r", "w_o", "w_4"):
                a[name] = mont_arr(rnd(ng))
        for name in PK_RANDOM_COEFFS:
            if satisfying:
                c = mont_arr(evals[name])
                lib.or_ntt(vp(c), lg_n, 1, 0)  # coefficients of the n-domain evaluations
            else:
                c = rand_fr_mont_arr(rng, n)
            e = np.zeros((N8, 4), dtype=np.uint64)
            lib.or_coset_lde8(vp(c), vp(e), lg_n)
            a[name + "_coeffs"] = c
            a[name + "_evals"] = e
        for name in PK_ZERO_EVALS:
            a[name] = np.zeros((N8, 4), dtype=np.uint64)
        if qm_qlookup_evals:
            # live q_m / q_lookup selectors (consistent coefficients + LDE)
            for sel in ("q_m", "q_lookup"):
                c = rand_fr_mont_arr(rng, n)
                e = np.zeros((N8, 4), dtype=np.uint64)
                lib.or_coset_lde8(vp(c), vp(e), lg_n)
                a[sel + "_coeffs"] = c
                a[sel + "_evals"] = e
        for t in ("table1", "table2", "table3", "table4"):
            a[t] = np.zeros((n, 4), dtype=np.uint64)
        if lookup_rows:
            # non-zero query rows; the table holds their wire tuples (so every
            # query is in the table, combine_split is defined), padded with
            # its first row (MultiSet::pad)
            rows = np.sort(rng.choice(ng, size=min(lookup_rows, ng), replace=False))
            a["q_lookup"][rows] = rand_fr_mont_arr(rng, len(rows))
            for j, (t, w) in enumerate(zip(("table1", "table2", "table3", "table4"),
                                           ("w_l", "w_r", "w_o", "w_4"))):
                col = a[w][rows[::-1]]
                a[t][:len(rows)] = col
                a[t][len(rows):] = col[0]
        # linear_evaluations = coset points g*w^i; v_h = (g w^i)^n - 1
        w8 = fr_root(lg_n + 3)
        xs, vh = [], []
        x = FR_GEN
        gn = pow(FR_GEN, n, R_MOD)
        w8n = pow(w8, n, R_MOD)
        vv = gn
        for i in range(N8):
            xs.append(fr_mont(x))
            vh.append(fr_mont((vv - 1) % R_MOD))
            x = x * w8 % R_MOD
            vv = vv * w8n % R_MOD
        a["linear_evaluations"] = ints_to_arr(xs)
        a["v_h_coset_8n"] = ints_to_arr(vh)
        # SRS: [tau^i] G for i < n, affine Montgomery
        tau = rand_fr_mont_arr(rng, 1)
        self.tau_mont = tau
        srs = np.zeros((n, 12), dtype=np.uint64)
        lib.or_srs(vp(srs), n, vp(tau))
        a["srs"] = srs
        a["gamma_g"] = np.zeros((2, 12), dtype=np.uint64)
        a["empty"] = np.zeros((1, 4), dtype=np.uint64)
        self._build_structs()

    def _build_structs(self):
        a = self.arrays
        self.circuit = abi.CircuitC(
            n=self.n_gates, lookup_len=0, intended_pi_pos=self.pi_pos,
            q_lookup=ptr_of(a["q_lookup"]), pi=ptr_of(a["pi"]), w_l=ptr_of(a["w_l"]),
            w_r=ptr_of(a["w_r"]), w_o=ptr_of(a["w_o"]), w_4=ptr_of(a["w_4"]))
        pk = abi.ProverKeyC()
        for f in abi.PK_FIELDS:
            key = f if f in a else None
            if key is None:
                # empty coeff vectors (q_m, custom selectors, q_lookup)
                key = "empty"
            setattr(pk, f, ptr_of(a[key]))
        self.pk = pk
        self.ck = abi.CommitKeyC(powers_of_g=ptr_of(a["srs"]), powers_of_gamma_g=ptr_of(a["gamma_g"]))

    def oracle_proof(self) -> abi.ProofC:
        lib = oracle()
        out = abi.ProofC()
        rc = lib.or_gen_proof(C.byref(self.circuit), C.byref(self.pk), C.byref(self.ck), C.byref(out))
        assert rc == 0, rc
        return out


# ------------------------------------------------------------------ verifier
# or_verifier_key (oracle/pnp_oracle.h): n, g[12], then 23 commitments of 12 u64
VK_POLYS = ("q_m", "q_l", "q_r", "q_o", "q_4", "q_c", "q_hl", "q_hr", "q_h4", "q_arith",
            "range_selector", "logic_selector", "fixed_group_add_selector",
            "variable_group_add_selector", "left_sigma", "right_sigma", "out_sigma",
            "fourth_sigma", "q_lookup", "table1", "table2", "table3", "table4")
VK_WORDS = 1 + 12 + 12 * len(VK_POLYS)


def _sig_verifier(lib):
    if getattr(lib, "_vk_sig", False):
        return
    vp_ = C.c_void_p
    lib.or_verifier_key_from_coeffs.argtypes = [vp_, C.c_uint64, vp_, C.c_void_p * len(VK_POLYS)]
    lib.or_verify_kzg_points.argtypes = [vp_, vp_, C.c_char_p, C.c_uint64, vp_, vp_, vp_]
    lib.or_verify_kzg_points.restype = C.c_int
    lib.or_verify.argtypes = [vp_, vp_, C.c_char_p, C.c_uint64, vp_, vp_, vp_]
    lib.or_verify.restype = C.c_int
    lib._vk_sig = True


def verifier_key(coeffs: dict, n: int, srs: np.ndarray) -> np.ndarray:
    """Commitments to the preprocessed polynomials (the VerifierKey that
    Circuit::compile returns, circuit.rs:232-264); coeffs maps a VK_POLYS name
    to its n Montgomery coefficients, absent = the zero polynomial."""
    lib = oracle()
    _sig_verifier(lib)
    vk = np.zeros(VK_WORDS, dtype=np.uint64)
    keep = [np.ascontiguousarray(coeffs[k]) if k in coeffs else None for k in VK_POLYS]
    ptrs = (C.c_void_p * len(VK_POLYS))(*[C.c_void_p(a.ctypes.data) if a is not None else None
                                          for a in keep])
    lib.or_verifier_key_from_coeffs(vp(vk), n, vp(np.ascontiguousarray(srs)), ptrs)
    return vk


def verifier_key_tau(coeffs: dict, n: int, g_aff: np.ndarray, tau_mont) -> np.ndarray:
    """verifier_key from the SRS trapdoor: commit(p) = [p(tau)] G, one Horner
    evaluation + one scalar multiplication per polynomial (oracle
    or_verifier_key_tau); equal to verifier_key when srs_i = [tau^i] G."""
    lib = oracle()
    _sig_verifier(lib)
    if not getattr(lib, "_vk_tau_sig", False):
        lib.or_verifier_key_tau.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p,
                                            C.c_void_p * len(VK_POLYS), C.c_void_p]
        lib._vk_tau_sig = True
    vk = np.zeros(VK_WORDS, dtype=np.uint64)
    keep = [np.ascontiguousarray(coeffs[k]) if k in coeffs else None for k in VK_POLYS]
    ptrs = (C.c_void_p * len(VK_POLYS))(*[C.c_void_p(a.ctypes.data) if a is not None else None
                                          for a in keep])
    g = np.ascontiguousarray(np.asarray(g_aff, dtype=np.uint64).reshape(12))
    tau = np.ascontiguousarray(np.asarray(tau_mont, dtype=np.uint64).reshape(4))
    lib.or_verifier_key_tau(vp(vk), n, vp(g), ptrs, vp(tau))
    return vk


def _pi_args(pis):
    pos = np.array([p for p, _ in pis], dtype=np.uint64)
    vals = np.array([to_limbs(v, 4) for _, v in pis], dtype=np.uint64).reshape(-1, 4)
    return pos, vals


def verify(vk: np.ndarray, proof: abi.ProofC, pis, tau_mont, label=b"Merkle tree") -> bool:
    """Oracle verifier (proof.rs:123-431) deciding the KZG checks with the SRS
    trapdoor tau; pis = [(pos, canonical value)]."""
    lib = oracle()
    _sig_verifier(lib)
    pos, vals = _pi_args(pis)
    tau = np.ascontiguousarray(np.asarray(tau_mont, dtype=np.uint64).reshape(4))
    return lib.or_verify(vp(vk), C.byref(proof), label, len(pis), vp(pos), vp(vals), vp(tau)) == 1


def kzg_points(vk: np.ndarray, proof: abi.ProofC, pis, label=b"Merkle tree"):
    """(L_aw, W_aw, L_saw, W_saw) affine: accept iff e(L, H) = e(W, [tau] H)."""
    lib = oracle()
    _sig_verifier(lib)
    pos, vals = _pi_args(pis)
    out = np.zeros((4, 12), dtype=np.uint64)
    rc = lib.or_verify_kzg_points(vp(vk), C.byref(proof), label, len(pis), vp(pos), vp(vals), vp(out))
    return rc, out


def inputs_vk(inp: "Inputs") -> np.ndarray:
    a = inp.arrays
    coeffs = {k: a[k + "_coeffs"] for k in VK_POLYS if k + "_coeffs" in a}
    return verifier_key(coeffs, inp.n, a["srs"])


def inputs_pis(inp: "Inputs"):
    return [(inp.pi_pos, from_limbs(inp.arrays["pi"]))]
