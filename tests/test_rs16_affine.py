"""The GF(2^16) encoder's layer constants are GF(2)-affine in the position bits above the layer.

rs16_kernels.hip writes a constant that depends on runtime wave bits as c_ct ^ w0*t5 ^ w1*t6 with compile-time
parts (c_ct from the register and specialised wave bits, t_i = g(2^i) ^ g(0)).  That holds because Leopard's FFT
skews are built as FFTSkew[j + 2^(i+1)] = FFTSkew[j] ^ temp[i] (klauspost/reedsolomon v1.12.1 leopardFF16
FFTInitialize), and field addition is XOR in every basis.  Checked here on the oracle's own
skew table (oracle/leopard.c), every layer and both transforms, for m = 512 (config C5) and m = 1024."""
import pytest

import oracle_lib as O


def _const(L, i):
    s = L.ora_leo_skew(16, i)
    return 0 if s >= 65535 else L.ora_leo_exp(16, s)  # log == modulus: no multiply (the zero element)


@pytest.mark.parametrize("log2m", [9, 10])
def test_layer_constants_affine_in_position_bits(log2m):
    L = O.lib()
    M = 1 << log2m
    for d in range(log2m):
        D = 1 << d
        for inverse in (False, True):
            def g(s0):
                return _const(L, (M - 1 + s0 + D) if inverse else (s0 + D - 1))
            base = g(0)
            t = {i: g(1 << i) ^ base for i in range(d + 1, log2m)}
            for s0 in range(0, M, 2 * D):
                acc = base
                for i, ti in t.items():
                    if (s0 >> i) & 1:
                        acc ^= ti
                assert acc == g(s0), (log2m, d, inverse, s0)
