"""The SHA-256 working state after the constant first 14 rounds of a parity inner node's first block (0x01 ‖ 0xFF x 58,
csrc/nmt_dev.h kParityMid14), recomputed here from FIPS 180-4, and the identity it relies on: finishing the
compression from that state equals the full compression for any last five bytes of the block."""
import os
import re
import struct

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
M32 = 0xFFFFFFFF
K = [0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98,
     0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786,
     0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8,
     0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13,
     0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819,
     0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a,
     0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
     0xc67178f2]
IV = [0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19]


def rotr(x, n):
    return ((x >> n) | (x << (32 - n))) & M32


def schedule(block):
    w = list(struct.unpack(">16I", block))
    for t in range(16, 64):
        s0 = rotr(w[t - 15], 7) ^ rotr(w[t - 15], 18) ^ (w[t - 15] >> 3)
        s1 = rotr(w[t - 2], 17) ^ rotr(w[t - 2], 19) ^ (w[t - 2] >> 10)
        w.append((w[t - 16] + s0 + w[t - 7] + s1) & M32)
    return w


def rounds(state, w, t0, t1):
    a, b, c, d, e, f, g, h = state
    for t in range(t0, t1):
        t1_ = (h + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g & M32)) + K[t] + w[t]) & M32
        t2_ = ((rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c))) & M32
        h, g, f, e, d, c, b, a = g, f, e, (d + t1_) & M32, c, b, a, (t1_ + t2_) & M32
    return [a, b, c, d, e, f, g, h]


def kernel_constant():
    src = open(os.path.join(ROOT, "celestia-app_amd", "csrc", "nmt_dev.h")).read()
    body = re.search(r"kParityMid14\[8\] = \{([^}]*)\}", src).group(1)
    return [int(x, 16) for x in re.findall(r"0x[0-9a-fA-F]+", body)]


def test_parity_midstate_constant():
    prefix = b"\x01" + b"\xff" * 58
    w = schedule(prefix + bytes(5))
    assert kernel_constant() == rounds(IV, w, 0, 14)


@pytest.mark.parametrize("seed", range(4))
def test_finishing_from_the_midstate_is_the_compression(seed):
    tail = os.urandom(5) if seed else bytes(5)
    w = schedule(b"\x01" + b"\xff" * 58 + tail)
    assert rounds(kernel_constant(), w, 14, 64) == rounds(IV, w, 0, 64)


def test_parity_leaf_midstate_constant():
    """kParityLeafMid7: a parity leaf's first block is 0x00 ‖ 0xFF x 29 ‖ share[0..34); rounds 0..6 are constant."""
    src = open(os.path.join(ROOT, "celestia-app_amd", "csrc", "nmt_dev.h")).read()
    body = re.search(r"kParityLeafMid7\[8\] = \{([^}]*)\}", src).group(1)
    mid = [int(x, 16) for x in re.findall(r"0x[0-9a-fA-F]+", body)]
    share_head = os.urandom(34)
    w = schedule(b"\x00" + b"\xff" * 29 + share_head)
    assert mid == rounds(IV, w, 0, 7)
    assert rounds(mid, w, 7, 64) == rounds(IV, w, 0, 64)
