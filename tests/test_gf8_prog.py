"""The g2 RS encoder multiplies by each FFT constant with a compile-time XOR3 program (csrc/gf8_const.h: the
constant's matrix in Leopard's own coordinates, shared terms factored out).  Host check of every program against
the oracle's Leopard multiply (oracle/leopard.c, klauspost/reedsolomon v1.12.1 mulLog8), byte by byte.  The GPU
parity tests check the same arithmetic end to end through the encoder."""
import os
import shutil
import subprocess

import pytest

import oracle_lib as O

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.fixture(scope="module")
def prog_lines(tmp_path_factory):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    exe = str(tmp_path_factory.mktemp("gf8") / "gf8_prog_check")
    subprocess.check_call([hipcc, "-O1", "-std=c++17", "--offload-arch=gfx950", "-o", exe,
                           os.path.join(ROOT, "tools", "gf8_prog_check.cpp")])
    out = subprocess.run([exe], capture_output=True, text=True, check=True, timeout=60)
    return out.stdout.split("\n")[:255]


def test_every_constant_program_matches_leopard_mul(prog_lines):
    L = O.lib()
    assert len(prog_lines) == 255
    for line in prog_lines:
        i, c, table = line.split()
        i, c = int(i), int(c)
        skew = L.ora_leo_skew(8, i)
        got = bytes.fromhex(table)
        if skew >= 255:  # log == modulus: the butterfly has no multiply
            assert c == 0
            continue
        e = L.ora_leo_exp(8, skew)
        want = bytes(L.ora_leo_mul(8, x, e) for x in range(256))
        assert got == want, f"skew index {i}"
