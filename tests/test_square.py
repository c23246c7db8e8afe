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


def _blob_tx(rng, nblobs):
    """A BlobTx (blob.MarshalBlobTx: tx=1, blobs=2, type_id=3 "BLOB") with random v0 namespaces and sizes."""
    tx = bytes(rng.integers(0, 256, int(rng.integers(50, 400)), dtype=np.uint8))
    out = b"\x0a" + S.varint(len(tx)) + tx
    for _ in range(nblobs):
        # v0 ID: 18 zero bytes then 10 bytes, above the reserved namespaces (first byte non-zero)
        ns_id = bytes(18) + bytes([int(rng.integers(1, 256))]) + bytes(rng.integers(0, 256, 9, dtype=np.uint8))
        data = bytes(rng.integers(0, 256, int(rng.integers(1, 6000)), dtype=np.uint8))
        blob = b"\x0a" + S.varint(len(ns_id)) + ns_id + b"\x12" + S.varint(len(data)) + data
        out += b"\x12" + S.varint(len(blob)) + blob
    return out + b"\x1a\x04BLOB"


def _random_txs(seed, n_normal, n_blob_txs):
    rng = np.random.default_rng(seed)
    txs = [bytes(rng.integers(0, 256, int(rng.integers(100, 900)), dtype=np.uint8)) for _ in range(n_normal)]
    txs += [_blob_tx(rng, int(rng.integers(1, 4))) for _ in range(n_blob_txs)]
    return txs


def test_plan_tiles_the_square():
    for seed in range(4):
        ss, segs, _ = S.plan(_random_txs(seed, 20, 15), 128, 64)
        assert segs[0]["first"] == 0 and sum(sg["n"] for sg in segs) == ss * ss
        assert all(a["first"] + a["n"] == b["first"] for a, b in zip(segs, segs[1:]))
        recs, data, reserved = S.device_plan(segs)
        for r, sg in zip(recs, segs):
            if sg["kind"] == "compact":
                assert S.compact_shares_needed(r.data_len) == sg["n"]


@pytest.mark.gpu
def test_device_square_mainnet_block_408(ctx):
    """cda_construct_extend_commit: block 408's plan assembled on the GPU gives the reference ODS and data_hash."""
    txs, data_hash = mainnet_txs()
    ss, segs, _ = S.plan(txs, 128, 64)
    ods, eds, rr, cr, dah = ctx.construct_extend_commit(ss, segs, want_ods=True)
    assert np.array_equal(ods, np.load(os.path.join(GOLDEN, "mainnet_h408.npz"))["ods"])
    assert dah == data_hash


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n_normal,n_blob", [(1, 0, 0), (2, 3, 0), (3, 0, 2), (4, 40, 30), (5, 200, 120)])
def test_device_square_matches_host(ctx, seed, n_normal, n_blob):
    """Random normal txs and multi-blob BlobTxs: the device-built ODS equals the host render byte for byte and the
    roots / DAH equal the oracle's on that ODS."""
    ss, segs, _ = S.plan(_random_txs(seed, n_normal, n_blob), 128, 64)
    host = np.frombuffer(b"".join(S.render(segs)), np.uint8).reshape(-1, 512)
    ods, eds, rr, cr, dah = ctx.construct_extend_commit(ss, segs, want_ods=True)
    assert np.array_equal(ods, host)
    rc, eds_o, rr_o, cr_o, dah_o = O.extend_commit(host)
    assert rc == 0 and dah == dah_o and np.array_equal(eds, eds_o)


def _recs_tuple(recs):
    return [(r.kind, r.first_share, r.nshares, r.share_version, r.data_off, r.data_len, r.reserved_off, bytes(r.ns))
            for r in recs]


@pytest.mark.parametrize("seed,n_normal,n_blob", [(408, None, None), (1, 40, 0), (2, 0, 6), (3, 25, 12)])
def test_segments_from_shares_reads_back_the_plan(seed, n_normal, n_blob):
    """go/cda SegmentsFromShares (mirrored by cda.square.segments_from_shares): reading the layout back from a
    constructed square gives exactly the planner's device plan -- records, payload and reserved bytes -- for mainnet
    block 408 and synthetic blocks of normal txs and multi-blob BlobTxs."""
    if seed == 408:
        txs, _ = mainnet_txs()
    else:
        txs = _random_txs(seed, n_normal, n_blob)
    ss, segs, _ = S.plan(txs, 128, 64)
    want = S.device_plan(segs)
    got = S.segments_from_shares(S.render(segs))
    assert _recs_tuple(got[0]) == _recs_tuple(want[0])
    assert np.array_equal(got[1], want[1]) and np.array_equal(got[2], want[2])
