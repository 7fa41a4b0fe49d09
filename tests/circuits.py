"""Satisfying general PLONK circuits for the parity tests of the lifted envelope.

A tiny composer over variables, enough to lay out rows that satisfy every gate
family the reference prover supports (plonk-core/src/proof_system/widget):

  * arithmetic  q_m ab + q_l a + q_r b + q_o c + q_4 d + q_hl a^5 + q_hr b^5
                + q_h4 d^5 + q_c + PI = 0                       (arithmetic.rs)
  * range       base-4 accumulator chain c = 4d + q, b = 4c + q, a = 4b + q,
                d_next = 4a + q, q in {0..3}                    (range.rs)
  * logic       quads a_next - 4a, b_next - 4b, d_next - 4d, c = product of
                the a and b quads, q_c = 1: AND, q_c = -1: XOR  (logic.rs)
  * fixed-base  one step of the Jubjub fixed-base scalar multiplication:
    scalar mul  (x_beta, y_beta) = (q_l, q_r), q_c = x_beta y_beta, bit in
                {-1, 0, 1} from d_next - 2d, c = bit q_c, accumulator
                (a, b) -> (a_next, b_next)                      (fixed_base_scalar_mul.rs)
  * curve add   (a, b) + (c, d) = (a_next, b_next), d_next = a d (curve_addition.rs)
  * lookup      q_lookup = 1 and the wires are a row of the 4-column table

Copy constraints are cycles over every slot holding the same variable
(sigma_j(i) = k_j' w^i' of the next slot, k = 1, 7, 13, 17, permutation/
constants.rs); padding rows are zero rows with identity sigmas.  The prover
key is built like Circuit::compile: selector / sigma coefficients = iNTT of
the row values, 8n evaluations = coset LDE, lookup table columns padded with
their first entry (MultiSet::pad).  Everything runs through the oracle's NTT
(test infrastructure), numbers are canonical Python ints until packed.

Jubjub (ark-ed-on-bls12-381, the embedded curve of the reference's ECC gates):
a = -1, d = -10240/10241 over Fr.
"""
import numpy as np

from pnp import abi
from pnp_testlib import (R_MOD, FR_GEN, fr_root, fr_mont, ints_to_arr, to_limbs, oracle, vp,
                         ptr_of, verifier_key)

JJ_A = R_MOD - 1
JJ_D = (-10240 * pow(10241, -1, R_MOD)) % R_MOD
K_COSET = (1, 7, 13, 17)
SEL = ("q_m", "q_l", "q_r", "q_o", "q_4", "q_c", "q_hl", "q_hr", "q_h4", "q_arith",
       "range_selector", "logic_selector", "fixed_group_add_selector",
       "variable_group_add_selector", "q_lookup")


def fr_sqrt(x: int):
    """Tonelli-Shanks in Fr (r - 1 = 2^32 t); None for a non-residue."""
    x %= R_MOD
    if x == 0:
        return 0
    if pow(x, (R_MOD - 1) // 2, R_MOD) != 1:
        return None
    s, t = 32, (R_MOD - 1) >> 32
    z = 7  # FR_GEN, a non-residue
    m, c, r_, b = s, pow(z, t, R_MOD), pow(x, (t + 1) // 2, R_MOD), pow(x, t, R_MOD)
    while b != 1:
        i, b2 = 0, b
        while b2 != 1:
            b2 = b2 * b2 % R_MOD
            i += 1
        c2 = pow(c, 1 << (m - i - 1), R_MOD)
        m, c, r_, b = i, c2 * c2 % R_MOD, r_ * c2 % R_MOD, b * c2 * c2 % R_MOD
    return r_


def jj_add(p, q):
    """Twisted Edwards addition (the curve_addition.rs equations)."""
    (x1, y1), (x2, y2) = p, q
    t = JJ_D * x1 * x2 * y1 * y2 % R_MOD
    x3 = (x1 * y2 + y1 * x2) * pow(1 + t, -1, R_MOD) % R_MOD
    y3 = (y1 * y2 - JJ_A * x1 * x2) * pow(1 - t, -1, R_MOD) % R_MOD
    return x3, y3


def jj_point(rng):
    """A random Jubjub point: y random, x^2 = (1 - y^2) / (a - d y^2)."""
    while True:
        y = int(rng.integers(2, 2**62))
        x2 = (1 - y * y) * pow((JJ_A - JJ_D * y * y) % R_MOD, -1, R_MOD) % R_MOD
        x = fr_sqrt(x2)
        if x is not None:
            return x, y


class Composer:
    def __init__(self, seed: int):
        self.rng = np.random.default_rng(seed)
        self.vals = [0]       # variable 0 = the constant zero
        self.rows = []        # (selectors dict, (va, vb, vc, vd))
        self.pis = {}         # row -> canonical value
        self.table = []       # rows of 4 canonical values

    def var(self, v: int) -> int:
        self.vals.append(v % R_MOD)
        return len(self.vals) - 1

    def rnd(self) -> int:
        return int.from_bytes(self.rng.bytes(32), "little") % R_MOD

    def row(self, sel, a=0, b=0, c=0, d=0):
        self.rows.append((dict(sel), (a, b, c, d)))
        return len(self.rows) - 1

    # ---- gate families
    def arith(self, a=None, b=None, d=None, q=None, pi=0, qm=True):
        """Random arithmetic gate over variables a, b, d (fresh when None); c solved."""
        q = dict(q or {})
        for k in ("q_l", "q_r", "q_o", "q_4", "q_c", "q_hl", "q_hr", "q_h4"):
            q.setdefault(k, self.rnd())
        q.setdefault("q_m", self.rnd() if qm else 0)
        q["q_arith"] = 1
        a = self.var(self.rnd()) if a is None else a
        b = self.var(self.rnd()) if b is None else b
        d = self.var(self.rnd()) if d is None else d
        va, vb, vd = self.vals[a], self.vals[b], self.vals[d]
        acc = (q["q_m"] * va * vb + q["q_l"] * va + q["q_r"] * vb + q["q_4"] * vd
               + q["q_hl"] * pow(va, 5, R_MOD) + q["q_hr"] * pow(vb, 5, R_MOD)
               + q["q_h4"] * pow(vd, 5, R_MOD) + q["q_c"] + pi) % R_MOD
        c = self.var((-acc) * pow(q["q_o"], -1, R_MOD))
        r = self.row(q, a, b, c, d)
        if pi:
            self.pis[r] = pi % R_MOD
        return r, (a, b, c, d)

    def range_chain(self, gates: int):
        """`gates` range rows + the row holding the final accumulator."""
        acc = 0
        d = self.var(acc)
        for _ in range(gates):
            q = [int(self.rng.integers(0, 4)) for _ in range(4)]
            c_v = 4 * acc + q[0]
            b_v = 4 * c_v + q[1]
            a_v = 4 * b_v + q[2]
            acc = 4 * a_v + q[3]
            self.row({"range_selector": 1}, self.var(a_v), self.var(b_v), self.var(c_v), d)
            d = self.var(acc)
        self.row({}, 0, 0, 0, d)

    def logic_chain(self, gates: int, xor: bool):
        a_v = b_v = d_v = 0
        rows = []
        for _ in range(gates):
            qa, qb = int(self.rng.integers(0, 4)), int(self.rng.integers(0, 4))
            qd = (qa ^ qb) if xor else (qa & qb)
            rows.append(((a_v, b_v, qa * qb, d_v), (qa, qb, qd)))
            a_v, b_v, d_v = 4 * a_v + qa, 4 * b_v + qb, 4 * d_v + qd
        for (a, b, w, d), _ in rows:
            self.row({"logic_selector": 1, "q_c": R_MOD - 1 if xor else 1},
                     self.var(a), self.var(b), self.var(w), self.var(d))
        self.row({}, self.var(a_v), self.var(b_v), 0, self.var(d_v))

    def fbsm_chain(self, gates: int):
        """Fixed-base steps: acc += bit * P_k with its own base per row."""
        acc = jj_point(self.rng)
        bits = 0
        for _ in range(gates):
            xb, yb = jj_point(self.rng)
            bit = int(self.rng.integers(-1, 2))
            xa, ya = (xb * bit) % R_MOD, (bit * bit * (yb - 1) + 1) % R_MOD
            self.row({"fixed_group_add_selector": 1, "q_l": xb, "q_r": yb, "q_c": xb * yb % R_MOD},
                     self.var(acc[0]), self.var(acc[1]), self.var(bit * xb * yb), self.var(bits))
            acc = jj_add(acc, (xa, ya))
            bits = 2 * bits + bit
        self.row({}, self.var(acc[0]), self.var(acc[1]), 0, self.var(bits))

    def curve_add(self):
        p1, p2 = jj_point(self.rng), jj_point(self.rng)
        p3 = jj_add(p1, p2)
        self.row({"variable_group_add_selector": 1}, self.var(p1[0]), self.var(p1[1]),
                 self.var(p2[0]), self.var(p2[1]))
        self.row({}, self.var(p3[0]), self.var(p3[1]), 0, self.var(p1[0] * p2[1]))

    def lookup_table(self, rows: int):
        self.table = [[self.rnd() for _ in range(4)] for _ in range(rows)]

    def lookup(self, k: int):
        t = self.table[k]
        return self.row({"q_lookup": 1}, *(self.var(v) for v in t))

    # ---- compile + witness
    def build(self, min_lg: int = 4):
        """Domain n = 2^lg >= rows + 1 (a zero row after the last gate, so no
        custom gate reads a wrapped "next" row); zero rows are appended as
        gates until the prover's domain next_pow2(max(gates, table rows)) is n."""
        n = 1 << min_lg
        while n < max(len(self.rows) + 1, len(self.table)):
            n <<= 1
        while len(self.rows) <= n // 2:
            self.row({})
        return GeneralInputs(self, n)


class GeneralInputs:
    """Same interface as pnp_testlib.Inputs (arrays, circuit/pk/ck structs,
    oracle_proof, vk) for a Composer circuit."""

    def __init__(self, cp: Composer, n: int):
        lib = oracle()
        self.n = n
        self.lg_n = n.bit_length() - 1
        lg = self.lg_n
        ng = len(cp.rows)
        self.n_gates = ng
        N8 = 8 * n
        w = fr_root(lg)
        wp = [pow(w, i, R_MOD) for i in range(n)]
        a = self.arrays = {}
        # witness (gate rows only; the prover pads with zeros)
        for j, name in enumerate(("w_l", "w_r", "w_o", "w_4")):
            a[name] = ints_to_arr([fr_mont(cp.vals[r[1][j]]) for r in cp.rows])
        a["q_lookup"] = ints_to_arr([fr_mont(r[0].get("q_lookup", 0)) for r in cp.rows])
        # sigmas: cycles over the slots of each variable
        slots = {}
        for i, (_, ws) in enumerate(cp.rows):
            for j, v in enumerate(ws):
                slots.setdefault(v, []).append((j, i))
        sig = [[K_COSET[j] * wp[i] % R_MOD for i in range(n)] for j in range(4)]
        for cyc in slots.values():
            for k, (j, i) in enumerate(cyc):
                j2, i2 = cyc[(k + 1) % len(cyc)]
                sig[j][i] = K_COSET[j2] * wp[i2] % R_MOD
        polys = {name: [r[0].get(name, 0) % R_MOD for r in cp.rows] + [0] * (n - ng) for name in SEL}
        for j, name in enumerate(("left_sigma", "right_sigma", "out_sigma", "fourth_sigma")):
            polys[name] = sig[j]
        self._sig = sig
        self.nonzero = set()
        for name, vals in polys.items():
            c = ints_to_arr([fr_mont(v) for v in vals])
            lib.or_ntt(vp(c), lg, 1, 0)
            e = np.zeros((N8, 4), dtype=np.uint64)
            lib.or_coset_lde8(vp(c), vp(e), lg)
            if any(vals):
                self.nonzero.add(name)
            # empty Rust Vec for the zero polynomial (never read by the prover)
            a[name + "_coeffs"] = c if (any(vals) or name in _ALWAYS) else np.zeros((1, 4), np.uint64)
            a[name + "_evals"] = e
        # lookup table columns, padded with their first entry (MultiSet::pad)
        tab = cp.table or [[0, 0, 0, 0]]
        for j in range(4):
            col = [row[j] for row in tab]
            col = col + [col[0]] * (n - len(col))
            a[f"table{j + 1}"] = ints_to_arr([fr_mont(v) for v in col])
            c = a[f"table{j + 1}"].copy()
            lib.or_ntt(vp(c), lg, 1, 0)
            a[f"table{j + 1}_coeffs"] = c
        self.lookup_len = len(cp.table)
        # coset points and Z_H on the 8n coset
        w8 = fr_root(lg + 3)
        xs, vh = [], []
        x, vv, w8n = FR_GEN, pow(FR_GEN, n, R_MOD), pow(w8, n, R_MOD)
        for _ in range(N8):
            xs.append(fr_mont(x))
            vh.append(fr_mont((vv - 1) % R_MOD))
            x = x * w8 % R_MOD
            vv = vv * w8n % R_MOD
        a["linear_evaluations"] = ints_to_arr(xs)
        a["v_h_coset_8n"] = ints_to_arr(vh)
        tau = ints_to_arr([fr_mont(cp.rnd())])
        self.tau_mont = tau
        srs = np.zeros((n, 12), dtype=np.uint64)
        lib.or_srs(vp(srs), n, vp(tau))
        a["srs"] = srs
        a["gamma_g"] = np.zeros((2, 12), dtype=np.uint64)
        self.pis = sorted(cp.pis.items())
        if not self.pis:
            self.pis = [(0, 0)]
        a["pi"] = np.array(to_limbs(self.pis[0][1], 4), dtype=np.uint64)
        self.pi_pos = self.pis[0][0]
        self._build_structs()

    @property
    def sigma_evals(self):
        """The 4 sigma polynomials on the n-domain (Montgomery arrays)."""
        return [ints_to_arr([fr_mont(v) for v in col]) for col in self._sig]

    def _build_structs(self):
        a = self.arrays
        self.circuit = abi.CircuitC(
            n=self.n_gates, lookup_len=self.lookup_len, intended_pi_pos=self.pi_pos,
            q_lookup=ptr_of(a["q_lookup"]), pi=ptr_of(a["pi"]), w_l=ptr_of(a["w_l"]),
            w_r=ptr_of(a["w_r"]), w_o=ptr_of(a["w_o"]), w_4=ptr_of(a["w_4"]))
        pk = abi.ProverKeyC()
        for f in abi.PK_FIELDS:
            setattr(pk, f, ptr_of(a[f]))
        self.pk = pk
        self.ck = abi.CommitKeyC(powers_of_g=ptr_of(a["srs"]), powers_of_gamma_g=ptr_of(a["gamma_g"]))

    def pi_args(self):
        pos = np.array([p for p, _ in self.pis], dtype=np.uint64)
        vals = np.array([to_limbs(v, 4) for _, v in self.pis], dtype=np.uint64).reshape(-1, 4)
        return pos, vals

    def oracle_proof(self, label: bytes = b"Merkle tree") -> abi.ProofC:
        import ctypes as C
        lib = oracle()
        out = abi.ProofC()
        pos, vals = self.pi_args()
        lib.or_gen_proof_ex.argtypes = [C.c_void_p] * 3 + [C.c_uint64, C.c_void_p, C.c_void_p,
                                                          C.c_char_p, C.c_void_p]
        lib.or_gen_proof_ex.restype = C.c_int
        rc = lib.or_gen_proof_ex(C.byref(self.circuit), C.byref(self.pk), C.byref(self.ck), len(pos),
                                 vp(pos), vp(vals), label, C.byref(out))
        assert rc == 0, rc
        return out

    def vk(self):
        a = self.arrays
        coeffs = {}
        for k in SEL + ("left_sigma", "right_sigma", "out_sigma", "fourth_sigma"):
            if k in self.nonzero or k in _ALWAYS:
                coeffs[k] = a[k + "_coeffs"]
        for j in range(4):
            coeffs[f"table{j + 1}"] = a[f"table{j + 1}_coeffs"]
        return verifier_key(coeffs, self.n, a["srs"])


# coefficient vectors the reference always passes in full (lib.rs:157-223)
_ALWAYS = {"q_l", "q_r", "q_o", "q_4", "q_c", "q_hl", "q_hr", "q_h4", "q_arith",
           "left_sigma", "right_sigma", "out_sigma", "fourth_sigma"}
