"""ctypes mirror of include/pnp_plonk.h.

This is the Python-side equivalent of the Rust FFI declarations in
plonk-core/src/lib.rs:52-239 (the structs are repr(C) there and plain C
structs here, field for field).  The host program (tests, bench) uses it to
marshal CircuitC / ProverKeyC / CommitKeyC exactly like Prover::prove_pnp
(plonk-core/src/proof_system/prover.rs:693-907) does on the Rust side.
"""
import ctypes as C

U64P = C.POINTER(C.c_uint64)
FR4 = C.c_uint64 * 4


class WireEvaluationsC(C.Structure):
    _fields_ = [("a_eval", FR4), ("b_eval", FR4), ("c_eval", FR4), ("d_eval", FR4)]


class PermutationEvaluationsC(C.Structure):
    _fields_ = [("left_sigma_eval", FR4), ("right_sigma_eval", FR4),
                ("out_sigma_eval", FR4), ("permutation_eval", FR4)]


class CustomEvaluationsC(C.Structure):
    _fields_ = [(n, FR4) for n in (
        "q_arith_eval", "q_c_eval", "q_l_eval", "q_r_eval", "q_hl_eval",
        "q_hr_eval", "q_h4_eval", "a_next_eval", "b_next_eval", "d_next_eval")]


class LookupEvaluationsC(C.Structure):
    _fields_ = [(n, FR4) for n in (
        "q_lookup_eval", "z2_next_eval", "h1_eval", "h1_next_eval", "h2_eval",
        "f_eval", "table_eval", "table_next_eval")]


class ProofEvaluationsC(C.Structure):
    _fields_ = [("wire_evals", WireEvaluationsC), ("perm_evals", PermutationEvaluationsC),
                ("lookup_evals", LookupEvaluationsC), ("custom_evals", CustomEvaluationsC)]


class CommitmentC(C.Structure):
    _fields_ = [("x", C.c_uint64 * 6), ("y", C.c_uint64 * 6)]


PROOF_COMMITMENTS = ("a_comm", "b_comm", "c_comm", "d_comm", "z_comm", "f_comm",
                     "h_1_comm", "h_2_comm", "z_2_comm", "t_1_comm", "t_2_comm",
                     "t_3_comm", "t_4_comm", "t_5_comm", "t_6_comm", "t_7_comm",
                     "t_8_comm", "aw_opening", "saw_opening")


class ProofC(C.Structure):
    _fields_ = [(n, CommitmentC) for n in PROOF_COMMITMENTS] + [
        ("evaluations", ProofEvaluationsC)]


class CircuitC(C.Structure):
    _fields_ = [("n", C.c_uint64), ("lookup_len", C.c_uint64), ("intended_pi_pos", C.c_uint64),
                ("q_lookup", U64P), ("pi", U64P), ("w_l", U64P), ("w_r", U64P),
                ("w_o", U64P), ("w_4", U64P)]


PK_FIELDS = (
    "q_m_coeffs", "q_m_evals", "q_l_coeffs", "q_l_evals", "q_r_coeffs", "q_r_evals",
    "q_o_coeffs", "q_o_evals", "q_4_coeffs", "q_4_evals", "q_c_coeffs", "q_c_evals",
    "q_hl_coeffs", "q_hl_evals", "q_hr_coeffs", "q_hr_evals", "q_h4_coeffs", "q_h4_evals",
    "q_arith_coeffs", "q_arith_evals",
    "range_selector_coeffs", "range_selector_evals",
    "logic_selector_coeffs", "logic_selector_evals",
    "fixed_group_add_selector_coeffs", "fixed_group_add_selector_evals",
    "variable_group_add_selector_coeffs", "variable_group_add_selector_evals",
    "q_lookup_coeffs", "q_lookup_evals", "table1", "table2", "table3", "table4",
    "left_sigma_coeffs", "left_sigma_evals", "right_sigma_coeffs", "right_sigma_evals",
    "out_sigma_coeffs", "out_sigma_evals", "fourth_sigma_coeffs", "fourth_sigma_evals",
    "linear_evaluations", "v_h_coset_8n")


class ProverKeyC(C.Structure):
    _fields_ = [(n, U64P) for n in PK_FIELDS]


class CommitKeyC(C.Structure):
    _fields_ = [("powers_of_g", U64P), ("powers_of_gamma_g", U64P)]


class AffineLayout(C.Structure):
    """pnp_affine_layout: where x, y (6 u64 Montgomery limbs each) and the
    infinity byte sit in one arkworks G1Affine of `stride` bytes."""
    _fields_ = [("stride", C.c_uint64), ("x_off", C.c_uint64), ("y_off", C.c_uint64),
                ("inf_off", C.c_uint64)]


# ark-ec 0.3 GroupAffine<g1::Parameters> as rustc lays it out on x86-64
# (x: Fp384, y: Fp384, infinity: bool, 7 bytes of padding)
ARK_G1_AFFINE = AffineLayout(stride=104, x_off=0, y_off=48, inf_off=96)

assert C.sizeof(ProofC) == 2656
assert C.sizeof(CircuitC) == 72
assert C.sizeof(ProverKeyC) == 44 * 8
assert C.sizeof(CommitKeyC) == 16


def proof_to_bytes(p: ProofC) -> bytes:
    return bytes(C.string_at(C.addressof(p), C.sizeof(p)))


def ptr(addr: int):
    """Raw integer address (host or HBM) -> uint64_t* for the structs."""
    return C.cast(C.c_void_p(addr), U64P)
