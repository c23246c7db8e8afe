"""Known-answer inputs/outputs taken from the reference's own tests.

pkg/da/data_availability_header_test.go:
  :15-25  nil / empty DAH hash = SHA256("")
  :27-32  MinDataAvailabilityHeader (k=1 tail padding share)
  :34-68  "typical" k=2 and "max square size" k=128 constant squares from
          generateShares (:247-263): namespace v0 with ID 0x00*18 ‖ 0x01*10,
          followed by 0xFF*483.
"""
import numpy as np

EMPTY_HASH = bytes.fromhex("e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855")
MIN_DAH = bytes.fromhex("3d96b7d238e7e0456f6af8e7cdf0a67bd6cf9c2089ecb559c659dcaa1f880353")
TYPICAL_K2 = bytes.fromhex("b56e4d251ac266f4b91cc5464b3fc7efcbdc888064647496d13133f0dc65ac25")
MAX_K128 = bytes.fromhex("0bd3abeeacfbb0b92dfbdac4a154868e3c4e79666f7fcf6c620bb90dd3a0dcf0")


def tail_padding_share():
    s = np.zeros(512, np.uint8)
    s[:28] = 0xFF
    s[28] = 0xFE
    s[29] = 0x01
    return s


def generate_shares(count):
    """data_availability_header_test.go:247-263 (all shares identical, hence sorted)."""
    s = np.zeros(512, np.uint8)
    s[19:29] = 0x01
    s[29:] = 0xFF
    return np.tile(s, (count, 1))
