"""Square construction (go-square square.Construct mirror, cda/square.py) pinned on mainnet block 408.

The block's raw txs (tests/golden/mainnet_h408_txs.npz, from the reference fixture
x/blob/test/testdata/block_response.json) must construct the square whose DAH is the
block header's data_hash: CPU through the oracle, GPU through libcda.
"""
import os

import numpy as np
import pytest

import oracle_lib as O
from cda import square as S

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def mainnet_txs():
    z = np.load(os.path.join(GOLDEN, "mainnet_h408_txs.npz"))
    offs = z["offsets"]
    return [z["data"][offs[i]:offs[i + 1]].tobytes() for i in range(len(offs) - 1)], z["data_hash"].tobytes()


def test_construct_mainnet_block_408():
    txs, data_hash = mainnet_txs()
    ss, shares, info = S.construct(txs, 128, 64)
    assert ss == 32 and len(shares) == 32 * 32
    assert info["blobs"] == 1 and info["normal_txs"] + info["pfbs"] == len(txs) == 274
    ods = np.frombuffer(b"".join(shares), np.uint8).reshape(-1, 512)
    assert np.array_equal(ods, np.load(os.path.join(GOLDEN, "mainnet_h408.npz"))["ods"])
    rc, _, _, _, dah = O.extend_commit(ods, want_eds=False)
    assert rc == 0 and dah == data_hash


def test_construct_errors_and_small_squares():
    txs, _ = mainnet_txs()
    with pytest.raises(S.SquareError):
        S.construct(txs, 16, 64)  # needs k = 32
    ss, shares, info = S.construct([], 128, 64)
    assert ss == 1 and shares == [S.padding_share(S.TAIL_PADDING_NAMESPACE)]
    ss, shares, _ = S.construct([b"\x01" * 1000], 128, 64)
    assert ss == 2 and shares[0][:29] == S.TX_NAMESPACE and shares[-1][:29] == S.TAIL_PADDING_NAMESPACE


def test_blob_tx_round_trip():
    from cda.inclusion import sparse_shares_needed
    ns = bytes(19) + bytes(range(10))
    blob = b"\x0a" + S.varint(28) + ns[1:] + b"\x12" + S.varint(3) + b"abc"
    raw = b"\x0a" + S.varint(5) + b"hello" + b"\x12" + S.varint(len(blob)) + blob + b"\x1a\x04BLOB"
    tx, blobs = S.unmarshal_blob_tx(raw)
    assert tx == b"hello" and blobs == [{"ns": ns, "data": b"abc", "share_version": 0}]
    assert S.unmarshal_blob_tx(b"\x01\x02") is None
    ss, shares, info = S.construct([raw], 128, 64)
    assert info["pfb_share_indexes"] == [[info["first_blob"]]]
    start = info["first_blob"]
    assert shares[start:start + sparse_shares_needed(3)] == S.sparse_shares(ns, b"abc")


@pytest.mark.gpu
def test_construct_and_extend_on_gpu(ctx):
    from cda import da
    txs, data_hash = mainnet_txs()
    _, shares, _ = S.construct(txs, 128, 64)
    assert da.new_data_availability_header(da.extend_shares(shares)).hash() == data_hash
