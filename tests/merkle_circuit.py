"""The reference's own circuit: the Poseidon Merkle tree of merkle-tree/ at any
HEIGHT, laid out row for row like the reference composer (test input for the
parity tests; circuit construction itself is out of scope for the product).

Restated from `/root/reference/Prize 1B/`:
  * Poseidon constants (plonk-hashing/src/poseidon/constants.rs:26-78):
      - round numbers: calc_round_numbers(t, true)     round_numbers.rs:50-98
      - round constants: Grain LFSR, 80-bit seed        round_constant.rs:12-169
        (field 1, sbox 1, 255 bits, t, R_F, R_P; each 32-byte draw read
        big-endian -> reversed -> ark-ff 0.3 `from_random_bytes`: little-endian
        integer with bit 255 masked, rejected when >= r)
      - MDS: Cauchy matrix 1 / (x_i + y_j), x = 0..t, y = t..2t   mds.rs:41-62
      - domain tag 2^arity - 1
  * native hash (poseidon_ref.rs:21-238, NativeSpecRef); a tree node is
    hash(left, right) with state [tag, left, right] (merkle-tree/src/lib.rs:
    25-39: the third input overflows the width-3 buffer and is dropped)
  * the constraint gadget (zprize_constraints.rs:141-262, PlonkSpecZZ): 3 addi
    rows, then 3 rows per round with the next round's keys pre-added through
    q_c: full rounds = full_affine_transform_gate (hash.rs:20-64: q_hl, q_hr,
    q_h4 = MDS row, q_o = -1), partial rounds = partial_affine_transform_gate
    (hash.rs:73-117: q_hl, q_r, q_4); + assert_equal (composer.rs:355-367)
    = 193 rows per hash
  * StandardComposer::new (composer.rs:210-249): zero variable constrained to
    0 (one poly_gate), 3 blinding rows (composer.rs:604-685)
  * MerkleTree::gen_constraints (merkle-tree/src/constraints.rs:20-107): the
    bottom non-leaf level over the leaves, the upper levels bottom-up, the
    root gate with PI = -root
HEIGHT = 15: 193 * (2^14 - 1) + 5 = 3,161,924 rows, the headline gate count.

Parity status of the constants: the reference holds no Poseidon output
vectors, so the Grain constants are pinned only through the reference's
round-number table (round_numbers.rs:110-135) and the gadget == native hash
check of zprize_constraints.rs:388-433; proofs are pinned by the verifier
like every other circuit (tests/test_general.py).
"""
from circuits import Composer, R_MOD
from poseidon import (PoseidonConstants, calc_round_numbers, poseidon_hash,  # noqa: F401
                      generate_round_constants, flat_constants)


# ---------------------------------------------------------------- composer
class MerkleComposer(Composer):
    """Composer rows in the reference's order; variable 0 is zero_var."""

    def __init__(self, seed: int):
        super().__init__(seed)
        # StandardComposer::with_expected_size: zero_var constrained to 0
        self.poly_gate(0, 0, 0, q_l=1)
        # add_blinding_factors: two random rows, then (r1, r2, 0, 0)
        r1 = r2 = 0
        self.blind = []  # the 8 blinding values (pnp_synth_merkle's d_blind)
        for _ in range(2):
            r1, r2 = self.var(self.rnd()), self.var(self.rnd())
            r3, r4 = self.var(self.rnd()), self.var(self.rnd())
            self.blind += [self.vals[v] for v in (r1, r2, r3, r4)]
            self.row({}, r1, r2, r3, r4)
        self.row({}, r1, r2, 0, 0)

    def poly_gate(self, a, b, c, q_m=0, q_l=0, q_r=0, q_o=0, q_c=0, pi=None):
        """composer.rs:280-328 (w_4 = zero_var)."""
        r = self.row({"q_m": q_m, "q_l": q_l, "q_r": q_r, "q_o": q_o, "q_c": q_c, "q_arith": 1},
                     a, b, c, 0)
        if pi is not None:
            self.pis[r] = pi % R_MOD
        return r

    def arithmetic_gate(self, a, b, c=None, q_m=0, q_l=0, q_r=0, q_o=R_MOD - 1, q_c=0, q_4=0, d=0,
                        pi=None):
        """arithmetic.rs:103-173: c solved when not given."""
        if c is None:
            va, vb, vd = self.vals[a], self.vals[b], self.vals[d]
            s = (q_m * va * vb + q_l * va + q_r * vb + q_c + q_4 * vd + (pi or 0)) * (-q_o)
            c = self.var(s)
        r = self.row({"q_m": q_m, "q_l": q_l, "q_r": q_r, "q_o": q_o, "q_c": q_c, "q_4": q_4,
                      "q_arith": 1}, a, b, c, d)
        if pi is not None:
            self.pis[r] = pi % R_MOD
        return c

    def assert_equal(self, a, b):
        self.poly_gate(a, b, 0, q_l=1, q_r=R_MOD - 1)

    def full_affine(self, x, sel):
        """hash.rs:20-64"""
        v = [self.vals[i] for i in x]
        w4 = (sel[0] * pow(v[0], 5, R_MOD) + sel[1] * pow(v[1], 5, R_MOD) + sel[2] * pow(v[2], 5, R_MOD)
              + sel[3]) * pow(-sel[4] % R_MOD, -1, R_MOD)
        w = self.var(w4)
        self.row({"q_hl": sel[0], "q_hr": sel[1], "q_h4": sel[2], "q_c": sel[3], "q_o": sel[4],
                  "q_arith": 1}, x[0], x[1], w, x[2])
        return w

    def partial_affine(self, x, sel):
        """hash.rs:73-117"""
        v = [self.vals[i] for i in x]
        w4 = (sel[0] * pow(v[0], 5, R_MOD) + sel[1] * v[1] + sel[2] * v[2] + sel[3]) \
            * pow(-sel[4] % R_MOD, -1, R_MOD)
        w = self.var(w4)
        self.row({"q_hl": sel[0], "q_r": sel[1], "q_4": sel[2], "q_c": sel[3], "q_o": sel[4],
                  "q_arith": 1}, x[0], x[1], w, x[2])
        return w

    def hash_gadget(self, pc: PoseidonConstants, left: int, right: int) -> int:
        """PoseidonZZRef::output_hash over PlonkSpecZZ (zprize_constraints.rs:
        82-125, 141-262); returns the output variable."""
        t, rk, M = pc.width, pc.round_constants, pc.mds
        st = [self.var(pc.domain_tag), left, right]
        off = 0
        minus1 = R_MOD - 1

        def full_round(st, off):
            res = list(st)
            if off == 0:
                res = [self.arithmetic_gate(res[i], 0, q_l=1, q_c=rk[i]) for i in range(t)]
            nxt = [0, 0, 0] if len(rk) - off == t else rk[off + t:off + 2 * t]
            return [self.full_affine(res, [M[r][0], M[r][1], M[r][2], nxt[r], minus1]) for r in range(t)]

        def partial_round(st, off):
            return [self.partial_affine(st, [M[r][0], M[r][1], M[r][2], rk[off + t + r], minus1])
                    for r in range(t)]
        for _ in range(pc.half_full_rounds):
            st = full_round(st, off)
            off += t
        for _ in range(pc.partial_rounds):
            st = partial_round(st, off)
            off += t
        for _ in range(pc.half_full_rounds):
            st = full_round(st, off)
            off += t
        return st[1]


def merkle_tree(pc: PoseidonConstants, leaves):
    """MerkleTree::new_with_leaf_nodes (tree.rs:64-140): level-order non-leaf
    nodes, node i has children 2i+1, 2i+2 (util.rs:25-33)."""
    nl = len(leaves) - 1
    nodes = [0] * nl
    for i in range(nl - 1, -1, -1):
        l, r = 2 * i + 1, 2 * i + 2
        lv = leaves[l - nl] if l >= nl else nodes[l]
        rv = leaves[r - nl] if r >= nl else nodes[r]
        nodes[i] = poseidon_hash(pc, lv, rv)
    return nodes


def merkle_circuit(height: int, seed: int = 1, pc: PoseidonConstants = None, corrupt_node: int = None):
    """The reference's Merkle-tree circuit for `height` (2^(height-1) random
    leaves).  corrupt_node: index of a non-leaf node whose witness value is
    changed (an unsatisfied circuit, for negative tests)."""
    pc = pc or PoseidonConstants()
    cp = MerkleComposer(seed)
    leaves = cp.leaves = [cp.rnd() for _ in range(1 << (height - 1))]
    nodes = merkle_tree(pc, leaves)
    if corrupt_node is not None:
        nodes = list(nodes)
        nodes[corrupt_node] = (nodes[corrupt_node] + 1) % R_MOD
    leaf_vars = [cp.var(v) for v in leaves]
    node_vars = [cp.var(v) for v in nodes]
    # level start indices 0, 1, 3, 7, ... (constraints.rs:39-45)
    starts, idx = [], 0
    for _ in range(height - 1):
        starts.append(idx)
        idx = 2 * idx + 1
    start = starts.pop()
    upper = 2 * start + 1
    for i in range(start, upper):
        out = cp.hash_gadget(pc, leaf_vars[2 * i + 1 - upper], leaf_vars[2 * i + 2 - upper])
        cp.assert_equal(node_vars[i], out)
    for start in reversed(starts):
        for i in range(start, 2 * start + 1):
            out = cp.hash_gadget(pc, node_vars[2 * i + 1], node_vars[2 * i + 2])
            cp.assert_equal(node_vars[i], out)
    # root gate: root - root = 0 through the PI (constraints.rs:100-106)
    cp.arithmetic_gate(node_vars[0], 0, c=0, q_l=1, pi=-nodes[0] % R_MOD)
    return cp, nodes


def merkle_rows(height: int) -> int:
    return 193 * ((1 << (height - 1)) - 1) + 5


def gate_residuals(cp: Composer):
    """Rows whose arithmetic equation is not satisfied (check_circuit_satisfied
    for the selectors the Merkle circuit uses)."""
    bad = []
    for i, (q, (a, b, c, d)) in enumerate(cp.rows):
        if not q.get("q_arith"):
            continue
        va, vb, vc, vd = (cp.vals[x] for x in (a, b, c, d))
        g = lambda k: q.get(k, 0)
        s = (g("q_m") * va * vb + g("q_l") * va + g("q_r") * vb + g("q_o") * vc + g("q_4") * vd
             + g("q_hl") * pow(va, 5, R_MOD) + g("q_hr") * pow(vb, 5, R_MOD) + g("q_h4") * pow(vd, 5, R_MOD)
             + g("q_c") + cp.pis.get(i, 0)) % R_MOD
        if s:
            bad.append(i)
    return bad
