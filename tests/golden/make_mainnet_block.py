#!/usr/bin/env python3
"""Build the k=32 ODS of Celestia mainnet block 408 from the reference's fixture and pin it to data_hash.

Input: /root/reference/x/blob/test/testdata/block_response.json. This is the
reference's own test data, fetched there from the public API (see
x/blob/test/decode_blob_tx_test.go:64-70). It holds the block's 274 txs, its
square_size (32) and its data_hash, which is the DAH hash of the extended square.

The script arranges the txs into the original data square the way go-square's
square.Construct does. That package is not vendored, so the rules are restated
from the reference's specs and call sites:
  - txs are split into normal txs and BlobTxs. Blobs are sorted stably by
    namespace (test/util/malicious/out_of_order_builder.go:24-45,63-150 shows
    the builder and its Export, here without the malicious swap).
  - compact shares for TRANSACTION and PAY_FOR_BLOB hold varint-delimited units,
    sequence length and reserved bytes (specs/src/specs/shares.md:61-80).
  - sparse blob shares, namespace / reserved / tail padding (shares.md:31-122).
  - a blob starts at a multiple of SubTreeWidth (specs/src/specs/data_square_layout.md:47-60).
    SubtreeRootThreshold is 64 (pkg/appconsts/v1/app_consts.go:6).
  - the PFB share reservation assumes worst-case share indexes of
    SquareSizeUpperBound^2 = 128^2 (pkg/appconsts/v1/app_consts.go:5).
The oracle (oracle/liboracle.so) then extends the square and hashes the DAH.
That hash must equal the block's data_hash. A match pins the whole chain
bit-exactly on real, non-constant data: square layout, Leopard FF8 parity,
erasured NMT roots and the RFC-6962 DAH.

Outputs: tests/golden/mainnet_h408.npz, holding the ODS (1024 x 512 uint8) and
data_hash, and tests/golden/mainnet_h408_txs.npz, the block's raw txs. The square
rules live in the product's host mirror celestia-app_amd/cda/square.py. The fixture is data: a rearrangement of the reference's fixture
bytes. Run from the repo root: python tests/golden/make_mainnet_block.py
"""
import base64
import json
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))

SRC = "/root/reference/x/blob/test/testdata/block_response.json"
OUT = os.path.join(HERE, "mainnet_h408.npz")
TXS = os.path.join(HERE, "mainnet_h408_txs.npz")  # the block's raw txs (fixture data)

SHARE = 512
NS = 29
TX_NS = bytes(28) + b"\x01"
PFB_NS = bytes(28) + b"\x04"
RESERVED_PAD_NS = bytes(28) + b"\xff"
TAIL_PAD_NS = b"\xff" * 28 + b"\xfe"
FIRST_COMPACT = SHARE - NS - 1 - 4 - 4  # 474
CONT_COMPACT = SHARE - NS - 1 - 4  # 478
FIRST_SPARSE = SHARE - NS - 1 - 4  # 478
CONT_SPARSE = SHARE - NS - 1  # 482
SUBTREE_ROOT_THRESHOLD = 64
SQUARE_SIZE_UPPER_BOUND = 128


sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
from cda.square import construct as _construct  # noqa: E402
from cda.square import parse_fields, read_varint, unmarshal_blob_tx  # noqa: E402,F401
from cda.inclusion import sparse_shares_needed  # noqa: E402,F401


def construct(txs):
    """square.Construct at SquareSizeUpperBound 128, SubtreeRootThreshold 64 (app v1, block 408)."""
    ss, shares, info = _construct(txs, SQUARE_SIZE_UPPER_BOUND, SUBTREE_ROOT_THRESHOLD)
    return ss, np.frombuffer(b"".join(shares), np.uint8).reshape(ss * ss, SHARE), info


def main():
    d = json.load(open(SRC))
    blk = d["block"]
    txs = [base64.b64decode(t) for t in blk["data"]["txs"]]
    want = base64.b64decode(blk["header"]["data_hash"])
    ss, ods, info = construct(txs)
    print("square size", ss, "(block says", blk["data"]["square_size"], ")", info)
    import oracle_lib as O
    rc, eds, rr, cr, dah = O.extend_commit(ods)
    print("oracle rc", rc, "DAH", dah.hex())
    print("want      ", want.hex())
    ok = rc == 0 and dah == want
    print("MATCH" if ok else "MISMATCH")
    if ok:
        old = np.load(OUT) if os.path.exists(OUT) else None
        if old is None or not np.array_equal(old["ods"], ods):
            np.savez_compressed(OUT, ods=ods, data_hash=np.frombuffer(want, np.uint8),
                                square_size=np.array([ss]))
            print("wrote", os.path.relpath(OUT, ROOT), os.path.getsize(OUT), "bytes")
        offs = np.zeros(len(txs) + 1, np.uint64)
        offs[1:] = np.cumsum([len(t) for t in txs])
        np.savez_compressed(TXS, data=np.frombuffer(b"".join(txs), np.uint8), offsets=offs,
                            data_hash=np.frombuffer(want, np.uint8), square_size=np.array([ss]))
        print("wrote", os.path.relpath(TXS, ROOT), os.path.getsize(TXS), "bytes")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
