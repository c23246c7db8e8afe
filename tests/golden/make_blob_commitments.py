#!/usr/bin/env python3
"""Blob share commitments of Celestia mainnet block 408, from the reference's fixture.

Input: /root/reference/x/blob/test/testdata/block_response.json (the fixture behind
x/blob/test/decode_blob_tx_test.go). Every BlobTx in it carries its blobs and one
MsgPayForBlobs (proto/celestia/blob/v1/tx.proto:17-34). The submitter computed its
share_commitments with go-square's inclusion.CreateCommitment, the call the
reference re-checks in x/blob/types/blob_tx.go:97-105, and the block committed to
them (make_mainnet_block.py pins the block's data_hash).

For every blob the script records namespace, data, share version, the share index
the square layout gave it (make_mainnet_block.construct: the index the PFB's
IndexWrapper carries) and the commitment from the PFB. These are inputs and
expected outputs for the commitment parity tests (CreateCommitment, and
pkg/inclusion GetCommitment over the block's EDS).

Output: tests/golden/mainnet_h408_blobs.npz. Run from the repo root:
    python tests/golden/make_blob_commitments.py
"""
import base64
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_mainnet_block as M  # noqa: E402

OUT = os.path.join(HERE, "mainnet_h408_blobs.npz")
PFB_URL = "/celestia.blob.v1.MsgPayForBlobs"


def varints(fields, num):
    """Repeated uint32 field `num`, packed or not."""
    out = []
    for f, wt, v in fields:
        if f != num:
            continue
        if wt == 0:
            out.append(v)
        elif wt == 2:
            i = 0
            while i < len(v):
                x, i = M.read_varint(v, i)
                out.append(x)
    return out


def pfb_of(tx):
    """TxRaw{body_bytes=1} -> TxBody{messages=1} -> Any{type_url=1, value=2} -> MsgPayForBlobs."""
    body = next(v for f, wt, v in M.parse_fields(tx) if f == 1 and wt == 2)
    msgs = [v for f, wt, v in M.parse_fields(body) if f == 1 and wt == 2]
    assert len(msgs) == 1  # ValidateBlobTx: exactly one sdk.Msg (blob_tx.go:47-52)
    anyf = M.parse_fields(msgs[0])
    assert next(v for f, wt, v in anyf if f == 1).decode() == PFB_URL
    m = M.parse_fields(next(v for f, wt, v in anyf if f == 2))
    return {"namespaces": [v for f, wt, v in m if f == 2], "sizes": varints(m, 3),
            "commitments": [v for f, wt, v in m if f == 4], "share_versions": varints(m, 8)}


def main():
    d = json.load(open(M.SRC))
    txs = [base64.b64decode(t) for t in d["block"]["data"]["txs"]]
    ss, _, info = M.construct(txs)
    starts = info["pfb_share_indexes"]
    ns, datas, vers, st, com, nsh = [], [], [], [], [], []
    p = 0
    for raw in txs:
        bt = M.unmarshal_blob_tx(raw)
        if bt is None:
            continue
        tx, blobs = bt
        pfb = pfb_of(tx)
        assert len(pfb["commitments"]) == len(blobs)
        for j, b in enumerate(blobs):
            assert pfb["namespaces"][j] == b["ns"] and pfb["sizes"][j] == len(b["data"])
            ns.append(b["ns"])
            datas.append(b["data"])
            vers.append(b["share_version"])
            st.append(starts[p][j])
            com.append(pfb["commitments"][j])
            nsh.append(M.sparse_shares_needed(len(b["data"])))
        p += 1
    offs = np.zeros(len(datas) + 1, np.uint64)
    offs[1:] = np.cumsum([len(x) for x in datas])
    np.savez_compressed(OUT, namespaces=np.frombuffer(b"".join(ns), np.uint8).reshape(-1, 29),
                        data=np.frombuffer(b"".join(datas), np.uint8), offsets=offs,
                        share_versions=np.array(vers, np.uint8), starts=np.array(st, np.int64),
                        nshares=np.array(nsh, np.int64),
                        commitments=np.frombuffer(b"".join(com), np.uint8).reshape(-1, 32),
                        square_size=np.array([ss]))
    print(f"{len(datas)} blobs in {p} PFBs, {int(offs[-1])} data bytes, shares per blob {min(nsh)}..{max(nsh)}; "
          f"wrote {os.path.relpath(OUT)} ({os.path.getsize(OUT)} bytes)")


if __name__ == "__main__":
    main()
