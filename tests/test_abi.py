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
