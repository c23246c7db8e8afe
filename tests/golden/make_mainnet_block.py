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
data_hash. The fixture is data: a rearrangement of the reference's fixture
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


# ---- protobuf (wire format) ----------------------------------------------------------------
def varint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def read_varint(buf, i):
    shift = v = 0
    while True:
        b = buf[i]
        i += 1
        v |= (b & 0x7F) << shift
        shift += 7
        if not b & 0x80:
            return v, i


def parse_fields(buf):
    """-> list of (field, wiretype, value) or None if not a well-formed message."""
    out, i = [], 0
    try:
        while i < len(buf):
            key, i = read_varint(buf, i)
            f, wt = key >> 3, key & 7
            if wt == 0:
                v, i = read_varint(buf, i)
            elif wt == 2:
                n, i = read_varint(buf, i)
                if i + n > len(buf):
                    return None
                v, i = bytes(buf[i:i + n]), i + n
            elif wt == 1:
                v, i = bytes(buf[i:i + 8]), i + 8
            elif wt == 5:
                v, i = bytes(buf[i:i + 4]), i + 4
            else:
                return None
            if f == 0:
                return None
            out.append((f, wt, v))
    except IndexError:
        return None
    return out


def unmarshal_blob_tx(raw):
    """go-square blob.UnmarshalBlobTx: BlobTx{tx=1, blobs=2, type_id=3 == "BLOB"}."""
    fields = parse_fields(raw)
    if fields is None:
        return None
    tx, blobs, type_id = b"", [], b""
    for f, wt, v in fields:
        if f == 1 and wt == 2:
            tx = v
        elif f == 2 and wt == 2:
            blobs.append(v)
        elif f == 3 and wt == 2:
            type_id = v
    if type_id != b"BLOB" or not blobs:
        return None
    parsed = []
    for b in blobs:
        ns_id, data, share_version, ns_version = b"", b"", 0, 0
        for f, wt, v in parse_fields(b):
            if f == 1:
                ns_id = v
            elif f == 2:
                data = v
            elif f == 3:
                share_version = v
            elif f == 4:
                ns_version = v
        parsed.append({"ns": bytes([ns_version]) + ns_id, "data": data, "share_version": share_version})
    return tx, parsed


def index_wrapper(tx, share_indexes):
    """blob.IndexWrapper{tx=1, share_indexes=2 (packed uint32), type_id=3 "INDX"} (proto3 encoding)."""
    out = b"\x0a" + varint(len(tx)) + tx
    if share_indexes:
        packed = b"".join(varint(x) for x in share_indexes)
        out += b"\x12" + varint(len(packed)) + packed
    out += b"\x1a" + varint(4) + b"INDX"
    return out


# ---- share arithmetic ------------------------------------------------------------------------
def compact_shares_needed(seq_bytes):
    if seq_bytes == 0:
        return 0
    if seq_bytes <= FIRST_COMPACT:
        return 1
    return 1 + math.ceil((seq_bytes - FIRST_COMPACT) / CONT_COMPACT)


def sparse_shares_needed(n):
    if n == 0:
        return 0
    if n <= FIRST_SPARSE:
        return 1
    return 1 + math.ceil((n - FIRST_SPARSE) / CONT_SPARSE)


def round_up_pow2(v):
    p = 1
    while p < v:
        p <<= 1
    return p


def blob_min_square_size(share_count):
    return round_up_pow2(math.ceil(math.sqrt(share_count)))


def subtree_width(share_count, threshold):
    s = math.ceil(share_count / threshold)
    return min(round_up_pow2(s), blob_min_square_size(share_count))


def next_share_index(cursor, share_count, threshold):
    w = subtree_width(share_count, threshold)
    return ((cursor + w - 1) // w) * w


def compact_shares(ns, units):
    """Compact share sequence (shares.md "Transaction Shares")."""
    seq = b"".join(varint(len(u)) + u for u in units)
    starts, off = [], 0
    for u in units:
        starts.append(off)
        off += len(varint(len(u))) + len(u)
    n = compact_shares_needed(len(seq))
    shares, pos = [], 0
    for s in range(n):
        first = s == 0
        header = ns + bytes([1 if first else 0]) + (len(seq).to_bytes(4, "big") if first else b"")
        cap = FIRST_COMPACT if first else CONT_COMPACT
        data_start = len(header) + 4
        chunk_lo, chunk_hi = pos, pos + cap
        first_unit = next((st for st in starts if chunk_lo <= st < chunk_hi), None)
        reserved = 0 if first_unit is None else data_start + (first_unit - chunk_lo)
        body = seq[chunk_lo:chunk_hi]
        share = header + reserved.to_bytes(4, "big") + body
        shares.append(share + bytes(SHARE - len(share)))
        pos = chunk_hi
    return shares


def sparse_shares(ns, data, share_version):
    n = sparse_shares_needed(len(data))
    shares, pos = [], 0
    for s in range(n):
        first = s == 0
        header = ns + bytes([(share_version << 1) | (1 if first else 0)])
        if first:
            header += len(data).to_bytes(4, "big")
        cap = SHARE - len(header)
        share = header + data[pos:pos + cap]
        shares.append(share + bytes(SHARE - len(share)))
        pos += cap
    return shares


def padding_share(ns):
    share = ns + b"\x01" + bytes(4)
    return share + bytes(SHARE - len(share))


# ---- square.Construct ----------------------------------------------------------------------
def construct(txs):
    normal, pfbs, blobs = [], [], []
    for raw in txs:
        bt = unmarshal_blob_tx(raw)
        if bt is None:
            normal.append(raw)
            continue
        tx, bl = bt
        pidx = len(pfbs)
        pfbs.append({"tx": tx, "idx": [0] * len(bl)})
        for j, b in enumerate(bl):
            n = sparse_shares_needed(len(b["data"]))
            blobs.append({"blob": b, "pfb": pidx, "j": j, "n": n,
                          "max_pad": subtree_width(n, SUBTREE_ROOT_THRESHOLD) - 1})
    tx_seq = sum(len(varint(len(t))) + len(t) for t in normal)
    worst = SQUARE_SIZE_UPPER_BOUND * SQUARE_SIZE_UPPER_BOUND
    pfb_seq = sum(len(varint(len(w))) + len(w)
                  for w in (index_wrapper(p["tx"], [worst] * len(p["idx"])) for p in pfbs))
    tx_shares, pfb_reserved = compact_shares_needed(tx_seq), compact_shares_needed(pfb_seq)
    current = tx_shares + pfb_reserved + sum(b["n"] + b["max_pad"] for b in blobs)
    ss = blob_min_square_size(current)
    blobs.sort(key=lambda b: b["blob"]["ns"])  # stable: PFB priority order within a namespace
    non_reserved_start = tx_shares + pfb_reserved
    cursor = end_last = non_reserved_start
    blob_shares = []
    for i, b in enumerate(blobs):
        cursor = next_share_index(cursor, b["n"], SUBTREE_ROOT_THRESHOLD)
        if i == 0:
            non_reserved_start = cursor
        pad = cursor - end_last
        assert pad <= b["max_pad"]
        pfbs[b["pfb"]]["idx"][b["j"]] = cursor
        if i > 0:
            blob_shares += [padding_share(blobs[i - 1]["blob"]["ns"])] * pad
        blob_shares += sparse_shares(b["blob"]["ns"], b["blob"]["data"], b["blob"]["share_version"])
        cursor += b["n"]
        end_last = cursor
    txs_sh = compact_shares(TX_NS, normal)
    pfb_sh = compact_shares(PFB_NS, [index_wrapper(p["tx"], p["idx"]) for p in pfbs])
    assert len(pfb_sh) <= pfb_reserved
    square = txs_sh + pfb_sh
    if blob_shares:
        square += [padding_share(RESERVED_PAD_NS)] * (non_reserved_start - len(square))
        square += blob_shares
    square += [padding_share(TAIL_PAD_NS)] * (ss * ss - len(square))
    assert len(square) == ss * ss
    return ss, np.frombuffer(b"".join(square), np.uint8).reshape(ss * ss, SHARE), {
        "normal_txs": len(normal), "pfbs": len(pfbs), "blobs": len(blobs),
        "tx_shares": len(txs_sh), "pfb_shares": len(pfb_sh), "pfb_reserved": pfb_reserved,
        "first_blob": non_reserved_start if blobs else None, "current_size": current,
        "pfb_share_indexes": [p["idx"] for p in pfbs]}


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
        np.savez_compressed(OUT, ods=ods, data_hash=np.frombuffer(want, np.uint8),
                            square_size=np.array([ss]))
        print("wrote", os.path.relpath(OUT, ROOT), os.path.getsize(OUT), "bytes")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
