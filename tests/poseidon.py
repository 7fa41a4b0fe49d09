"""Poseidon (width 3) over BLS12-381 Fr as the reference's plonk-hashing crate
defines it: round numbers, Grain-LFSR round constants, Cauchy MDS, domain tag
(constants.rs:26-78) and the native hash (poseidon_ref.rs:21-238).  Shared by
tests/merkle_circuit.py (the circuit builder) and bench.py (which hands the
constants to pnp_synth_merkle); no oracle or GPU dependency.
"""
from collections import deque

R_MOD = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
WIDTH = 3
FIELD_BITS = 255


# ---------------------------------------------------------------- constants
def _rf_min(t: int, rp: int) -> int:
    """round_numbers.rs:82-98 in f32 like the reference (`rf >= rf_max` is
    secure; a negative bound casts to 0 as Rust's `as usize` saturates)."""
    import numpy as np
    f = np.float32
    n, m = f(256), f(128)
    rp_, t_ = f(rp), f(t)
    rf_stat = f(6.0) if m <= (n - f(3.0)) * (t_ + f(1.0)) else f(10.0)
    rf_interp = f(0.43) * m + np.log2(t_) - rp_
    rf_grob_1 = f(0.21) * n - rp_
    rf_grob_2 = (f(0.14) * n - f(1.0) - rp_) / (t_ - f(1.0))
    return max(max(int(np.ceil(v)), 0) for v in (rf_stat, rf_interp, rf_grob_1, rf_grob_2))


def calc_round_numbers(t: int, security_margin: bool = True):
    """round_numbers.rs:50-78: minimal t R_F + R_P over R_F even, R_P in
    4..200, then R_F + 2 and ceil(1.075 R_P) when security_margin."""
    import math
    import numpy as np
    rf = rp = 0
    best = None
    rf_min = {rp_test: _rf_min(t, rp_test) for rp_test in range(4, 200)}
    for rf_test in range(2, 1001, 2):
        for rp_test in range(4, 200):
            if rf_test < rf_min[rp_test]:
                continue
            rf2, rp2 = rf_test, rp_test
            if security_margin:
                rf2 += 2
                rp2 = int(math.ceil(np.float32(1.075) * np.float32(rp_test)))
            cost = t * rf2 + rp2
            if best is None or cost < best or (cost == best and rf2 < rf):
                rf, rp, best = rf2, rp2, cost
    return rf, rp


class _Grain:
    """GrainLFSR of round_constant.rs:84-169 (80-bit state, taps 62 51 38 23
    13 0, 160 discarded bits, bit pairs: keep the second bit when the first
    is 1)."""

    def __init__(self, field: int, sbox: int, field_size: int, t: int, r_f: int, r_p: int):
        bits = []

        def app(nb, v):
            bits.extend((v >> i) & 1 for i in range(nb - 1, -1, -1))
        app(2, field)
        app(4, sbox)
        app(12, field_size)
        app(12, t)
        app(10, r_f)
        app(10, r_p)
        app(30, (1 << 30) - 1)
        assert len(bits) == 80
        self.s = deque(bits)
        self.field_size = field_size
        for _ in range(160):
            self._new_bit()

    def _new_bit(self) -> int:
        s = self.s
        b = s[62] ^ s[51] ^ s[38] ^ s[23] ^ s[13] ^ s[0]
        s.popleft()
        s.append(b)
        return b

    def _next(self) -> int:
        b = self._new_bit()
        while not b:
            self._new_bit()
            b = self._new_bit()
        return self._new_bit()

    def _byte(self, nbits: int) -> int:
        acc = 0
        for _ in range(nbits):
            acc = (acc << 1) | self._next()
        return acc

    def next_bytes(self, n: int) -> bytes:
        rem = self.field_size % 8
        out = [self._byte(rem if rem else 8)]
        out += [self._byte(8) for _ in range(n - 1)]
        return bytes(out)


def generate_round_constants(t: int, r_f: int, r_p: int):
    g = _Grain(1, 1, FIELD_BITS, t, r_f, r_p)
    out = []
    while len(out) < (r_f + r_p) * t:
        be = g.next_bytes(32)
        v = int.from_bytes(be, "big")          # repr.reverse() + little-endian read
        v &= (1 << 255) - 1                    # ark-ff 0.3: REPR_SHAVE_BITS = 1
        if v < R_MOD:
            out.append(v)
    return out


class PoseidonConstants:
    def __init__(self, width: int = WIDTH):
        self.width = width
        self.full_rounds, self.partial_rounds = calc_round_numbers(width, True)
        self.half_full_rounds = self.full_rounds // 2
        self.round_constants = generate_round_constants(width, self.full_rounds, self.partial_rounds)
        self.mds = [[pow(i + j + width, -1, R_MOD) for j in range(width)] for i in range(width)]
        self.domain_tag = (1 << (width - 1)) - 1


# ---------------------------------------------------------------- native hash
def poseidon_hash(pc: PoseidonConstants, left: int, right: int) -> int:
    """PoseidonRef::output_hash over NativeSpecRef (poseidon_ref.rs:195-238)."""
    t, rk, M = pc.width, pc.round_constants, pc.mds
    st = [pc.domain_tag, left % R_MOD, right % R_MOD]
    off = 0

    def mds(s):
        return [sum(M[i][j] * s[i] for i in range(t)) % R_MOD for j in range(t)]

    def full(s, off):
        return mds([pow((s[i] + rk[off + i]) % R_MOD, 5, R_MOD) for i in range(t)])

    def partial(s, off):
        s = [(s[i] + rk[off + i]) % R_MOD for i in range(t)]
        s[0] = pow(s[0], 5, R_MOD)
        return mds(s)
    for _ in range(pc.half_full_rounds):
        st = full(st, off)
        off += t
    for _ in range(pc.partial_rounds):
        st = partial(st, off)
        off += t
    for _ in range(pc.half_full_rounds):
        st = full(st, off)
        off += t
    return st[1]


def flat_constants(pc: "PoseidonConstants"):
    """199 canonical ints for pnp_synth_merkle: round constants, MDS row-major, tag."""
    return list(pc.round_constants) + [pc.mds[j][i] for j in range(3) for i in range(3)] + [pc.domain_tag]
