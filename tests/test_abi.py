"""CPU-side checks of the C-ABI library: it loads, and exports every symbol
include/pnp_plonk.h declares (no compute calls: there is no GPU here)."""
import ctypes as C
import os
import re

from pnp_testlib import REPO


def _declared():
    src = open(os.path.join(REPO, "include", "pnp_plonk.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b((?:pnp_\w+|gen_proof))\s*\(", src)))


def test_library_exports_header_symbols():
    import pnp
    lib = pnp.load()
    declared = _declared()
    assert "gen_proof" in declared and len(declared) >= 18
    missing = [s for s in declared if not hasattr(lib, s)]
    assert missing == []
    assert set(declared) == set(pnp.SYMBOLS)


def test_struct_layouts():
    from pnp import abi
    assert C.sizeof(abi.ProofC) == 2656
    assert C.sizeof(abi.ProverKeyC) == 44 * 8
    assert C.sizeof(abi.CircuitC) == 72
    off = abi.ProofC.evaluations.offset
    assert off == 19 * 96


def test_proof_infinity_mask_host():
    """pnp_proof_infinity_mask (host code, no GPU): (0, Fq one) is infinity,
    (0, 2) is a finite curve point (y^2 = x^3 + 4), other points are finite;
    the bit order is ProofC's commitment order."""
    import pnp
    from pnp import abi
    from pnp_testlib import to_limbs, Q_MOD
    one = to_limbs((1 << 384) % Q_MOD, 6)
    two = to_limbs((2 << 384) % Q_MOD, 6)
    p = abi.ProofC()
    for k, name in enumerate(abi.PROOF_COMMITMENTS):
        c = getattr(p, name)
        c.x[0] = k + 1  # finite
        c.y[:] = two
    for name in ("f_comm", "h_1_comm", "h_2_comm", "t_7_comm", "t_8_comm"):
        c = getattr(p, name)
        c.x[:] = [0] * 6
        c.y[:] = one
    p.z_comm.x[:] = [0] * 6  # (0, 2): on the curve, not infinity
    m = pnp.infinity_mask(p)
    assert m == (1 << 5) | (1 << 6) | (1 << 7) | (1 << 15) | (1 << 16)
    flags = pnp.infinity_flags(p)
    assert [k for k, v in flags.items() if v] == ["f_comm", "h_1_comm", "h_2_comm", "t_7_comm", "t_8_comm"]


def test_ark_g1_affine_layout_shape():
    from pnp import abi
    L = abi.ARK_G1_AFFINE
    assert C.sizeof(abi.AffineLayout) == 32
    assert (L.stride, L.x_off, L.y_off, L.inf_off) == (104, 0, 48, 96)


def test_rccl_library_exports_header_symbols():
    """libpnp_rccl.so exports every function include/pnp_rccl.h declares.
    Checked in a child process that never imports torch (the library maps
    /opt/rocm's RCCL; a torch process keeps its own)."""
    import subprocess
    import sys
    src = open(os.path.join(REPO, "include", "pnp_rccl.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    declared = sorted(set(re.findall(r"\b(pnp_rccl_\w+)\s*\(", src)))
    assert len(declared) == 8, declared
    lib = os.path.join(REPO, "zprize23-gpu-submission_amd", "lib", "libpnp_rccl.so")
    code = ("import ctypes, sys; l = ctypes.CDLL(sys.argv[1]); "
            "print(' '.join(s for s in sys.argv[2:] if not hasattr(l, s)))")
    out = subprocess.run([sys.executable, "-c", code, lib] + declared, capture_output=True, text=True,
                         timeout=60)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "", f"missing: {out.stdout}"
