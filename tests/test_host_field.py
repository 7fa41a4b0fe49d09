"""The host half of csrc/field.cuh against Python integers.

The prover does its challenge arithmetic (round 5's linearisation scalars,
the Lagrange and vanishing values) and the commitments' affine conversion on
the host, between device round trips.  Those use the host paths of
field.cuh: a CIOS Montgomery product on 64-bit words and a binary extended
Euclidean inverse (mont_mul_host / inverse_host).  tests/native/host_field.cpp
prints seeded operands (zero, one, -1, the raw integer 1, P - 2 and random
residues) with a*b and inv(a); here each line is checked exactly:
a*b == a b R^-1 mod P and a * inv(a) == R^2 mod P (Montgomery forms), inv(0) = 0.
fr_inverse_bin (the device's batch-inverse base case, poly.hip k_inv_small)
is the same host/device source and is checked the same way.
The golden proofs on the GPU cover the same code end to end."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "zprize23-gpu-submission_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
MOD = {
    "r": (0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001, 256),
    "q": (0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab, 384),
}


@pytest.fixture(scope="module")
def lines(tmp_path_factory):
    if not (os.path.exists(HIPCC) or shutil.which("hipcc")):
        pytest.skip("hipcc not available")
    exe = str(tmp_path_factory.mktemp("hf") / "host_field")
    subprocess.run([HIPCC, "-O2", "-std=c++17", "--offload-host-only", "-x", "hip", "-I", CSRC,
                    os.path.join(HERE, "native", "host_field.cpp"), "-o", exe], check=True, timeout=300)
    out = subprocess.run([exe, "300"], check=True, capture_output=True, text=True, timeout=60).stdout
    return [ln.split() for ln in out.splitlines()]


@pytest.mark.parametrize("field", ["r", "q"])
def test_host_mont_product_and_inverse(lines, field):
    p, bits = MOD[field]
    R = 1 << bits
    rinv = pow(R, -1, p)
    rows = [ln[1:] for ln in lines if ln[0] == field]
    assert len(rows) == 300
    for a, b, ab, inv in ([int(x, 16) for x in row] for row in rows):
        assert a < p and b < p
        assert ab == a * b * rinv % p
        if a == 0:
            assert inv == 0
        else:
            assert inv < p and a * inv % p == R * R % p


def test_fr_inverse_bin(lines):
    p, bits = MOD["r"]
    R = 1 << bits
    rows = [[int(x, 16) for x in ln[1:]] for ln in lines if ln[0] == "b"]
    assert len(rows) == 300
    for a, inv in rows:
        if a == 0:
            assert inv == 0
        else:
            assert inv < p and a * inv % p == R * R % p
