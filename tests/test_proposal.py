"""ProcessProposal's BlobTx checks with a batched commitment pre-pass (cda/proposal.py, go/patches/0003):
ValidateBlobTx's checks and their order (x/blob/types/blob_tx.go:37-107), pinned on mainnet block 408's PFB
(x/blob/test/testdata/block_response.json via tests/golden/mainnet_h408_txs.npz) and on synthetic proposals whose
MsgPayForBlobs carry oracle-made commitments.  CPU tests inject the oracle as the commitment engine (a test double
for the parsing and check order); the GPU tests run the product path: ONE cda_blob_commitments call for the whole
proposal."""
import os

import numpy as np
import pytest

import oracle_lib as O
from cda import proposal as P
from cda import square as S

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def mainnet_txs():
    z = np.load(os.path.join(GOLDEN, "mainnet_h408_txs.npz"))
    offs = z["offsets"]
    return [z["data"][offs[i]:offs[i + 1]].tobytes() for i in range(len(offs) - 1)]


class OracleCommitments:
    """Test double with the context's blob_commitments signature, computed by the CPU oracle; counts calls."""

    def __init__(self):
        self.calls = 0

    def blob_commitments(self, namespaces, datas, share_versions=None, subtree_root_threshold=64):
        self.calls += 1
        out = []
        for i, (ns, d) in enumerate(zip(namespaces, datas)):
            rc, c = O.blob_commitment(bytes(ns), bytes(d), share_versions[i] if share_versions else 0,
                                      subtree_root_threshold)
            assert rc == 0
            out.append(c)
        return out


def _ld(field, payload):
    return S.varint(field << 3 | 2) + S.varint(len(payload)) + payload


def _uv(field, v):
    return S.varint(field << 3) + S.varint(v)


def pfb_blob_tx(blobs, commitments, signer=b"celestia1xyz", url=P.PFB_URL, sizes=None, extra_msg=False):
    """A BlobTx whose sdk tx carries one MsgPayForBlobs (tx.proto:17-34) over `blobs` = [(ns29, data)]."""
    msg = _ld(1, signer)
    for ns, _ in blobs:
        msg += _ld(2, ns)
    for i, (_, d) in enumerate(blobs):
        msg += _uv(3, len(d) if sizes is None else sizes[i])
    for c in commitments:
        msg += _ld(4, c)
    for _ in blobs:
        msg += _uv(8, 0)
    anyv = _ld(1, url) + _ld(2, msg)
    body = _ld(1, anyv) + (_ld(1, anyv) if extra_msg else b"")
    tx = _ld(1, body) + _ld(2, b"\x0a\x00") + _ld(3, b"sig")
    out = _ld(1, tx)
    for ns, d in blobs:
        out += _ld(2, _ld(1, ns[1:]) + _ld(2, d) + (_uv(4, ns[0]) if ns[0] else b""))
    return out + _ld(3, b"BLOB")


def random_proposal(seed, n_blob_txs=6, n_normal=5):
    rng = np.random.default_rng(seed)
    txs = [bytes(rng.integers(0, 256, int(rng.integers(100, 400)), dtype=np.uint8)) for _ in range(n_normal)]
    for _ in range(n_blob_txs):
        blobs = []
        for _ in range(int(rng.integers(1, 4))):
            ns = bytes(19) + bytes([int(rng.integers(1, 256))]) + bytes(rng.integers(0, 256, 9, dtype=np.uint8))
            blobs.append((ns, bytes(rng.integers(0, 256, int(rng.integers(1, 9000)), dtype=np.uint8))))
        txs.append(pfb_blob_tx(blobs, [O.blob_commitment(ns, d)[1] for ns, d in blobs]))
    order = rng.permutation(len(txs))
    return [txs[i] for i in order]


def test_mainnet_block_408_blob_tx_is_valid():
    txs = mainnet_txs()
    eng = OracleCommitments()
    assert P.process_proposal_blob_txs(txs, ctx=eng) == (None, None)
    assert eng.calls == 1  # the whole proposal's commitments in one call
    blob_idx = [i for i, t in enumerate(txs) if S.unmarshal_blob_tx(t) is not None]
    assert len(blob_idx) == 1
    # the PFB's commitment is the fixture's (make_blob_commitments.py read it from the same tx)
    z = np.load(os.path.join(GOLDEN, "mainnet_h408_blobs.npz"))
    tx, blobs = S.unmarshal_blob_tx(txs[blob_idx[0]])
    pfb = P.parse_pfb(P.decode_pfb_tx(tx)[0][1])
    assert pfb["share_commitments"] == [z["commitments"][0].tobytes()]
    assert pfb["blob_sizes"] == [len(blobs[0]["data"])]


def test_synthetic_proposal_valid_and_batched():
    txs = random_proposal(1)
    eng = OracleCommitments()
    assert P.process_proposal_blob_txs(txs, ctx=eng) == (None, None)
    assert eng.calls == 1


def _tamper(seed, which):
    rng = np.random.default_rng(seed)
    ns = bytes(19) + b"\x07" + bytes(rng.integers(0, 256, 9, dtype=np.uint8))
    d = bytes(rng.integers(0, 256, 3000, dtype=np.uint8))
    c = O.blob_commitment(ns, d)[1]
    if which == "commitment":
        return pfb_blob_tx([(ns, d)], [bytes(32)]), "ErrInvalidShareCommitment"
    if which == "size":
        return pfb_blob_tx([(ns, d)], [c], sizes=[2999]), "ErrBlobSizeMismatch"
    if which == "zero":
        return pfb_blob_tx([(ns, b"")], [c]), "ErrZeroBlobSize"
    if which == "reserved":
        rns = bytes(28) + b"\x01"
        return pfb_blob_tx([(rns, d)], [c]), "ErrReservedNamespace"
    if which == "no_pfb":
        return pfb_blob_tx([(ns, d)], [c], url=b"/cosmos.bank.v1beta1.MsgSend"), "ErrNoPFB"
    if which == "two_msgs":
        return pfb_blob_tx([(ns, d)], [c], extra_msg=True), "ErrMultipleMsgsInBlobTx"
    if which == "short_commitment":
        return pfb_blob_tx([(ns, d)], [c[:31]]), "ErrInvalidShareCommitment"
    if which == "ns_mismatch":
        other = bytes(19) + b"\x08" + ns[20:]
        tx = pfb_blob_tx([(ns, d)], [c])
        return tx.replace(ns, other, 1), "ErrNamespaceMismatch"  # the PFB's namespace (first copy) changes
    raise ValueError(which)


@pytest.mark.parametrize("which", ["commitment", "size", "zero", "reserved", "no_pfb", "two_msgs",
                                   "short_commitment", "ns_mismatch"])
def test_first_invalid_blob_tx_is_reported(which):
    txs = random_proposal(2)
    bad, code = _tamper(3, which)
    txs.insert(4, bad)
    eng = OracleCommitments()
    assert P.process_proposal_blob_txs(txs, ctx=eng) == (4, code)
    assert eng.calls <= 2  # the batch (+ one per-tx call only for a tx left out of the batch)


class FailingBatch(OracleCommitments):
    """The batch call fails (a device error); per-tx calls succeed."""

    def blob_commitments(self, namespaces, datas, share_versions=None, subtree_root_threshold=64):
        if self.calls == 0:
            self.calls += 1
            from cda import _native as N
            raise N.CdaError(-5, "injected batch failure")
        return super().blob_commitments(namespaces, datas, share_versions, subtree_root_threshold)


def test_failed_batch_falls_back_to_per_tx():
    txs = random_proposal(11)
    eng = FailingBatch()
    assert P.precompute_commitments(txs, ctx=eng) == [None] * len(txs)
    eng = FailingBatch()
    assert P.process_proposal_blob_txs(txs, ctx=eng) == (None, None)
    n_blob_txs = sum(S.unmarshal_blob_tx(t) is not None for t in txs)
    assert eng.calls == 1 + n_blob_txs


def test_batched_and_per_tx_agree():
    txs = random_proposal(5)
    eng = OracleCommitments()
    pre = P.precompute_commitments(txs, ctx=eng)
    for t, p in zip(txs, pre):
        if S.unmarshal_blob_tx(t) is None:
            assert p is None
            continue
        P.validate_blob_tx(t, precomputed=p, ctx=eng)
        P.validate_blob_tx(t, precomputed=None, ctx=eng)


class RecordingCommitments(OracleCommitments):
    """Records the namespaces of every blob handed to the batch call."""

    def __init__(self):
        super().__init__()
        self.batches = []

    def blob_commitments(self, namespaces, datas, share_versions=None, subtree_root_threshold=64):
        self.batches.append([bytes(n) for n in namespaces])
        return super().blob_commitments(namespaces, datas, share_versions, subtree_root_threshold)


@pytest.mark.parametrize("which", ["reserved", "zero"])
def test_blob_tx_rejected_by_validate_blobs_is_left_out_of_the_batch(which):
    """the batch holds exactly the BlobTxs whose blobs ValidateBlobs accepts (the Go pre-pass's filter):
    a reserved-namespace blob (and an empty one) stays out of the batched call, is checked on its own, and is reported
    at its index with the reference's error."""
    txs = random_proposal(21)
    bad, code = _tamper(22, which)
    txs.insert(3, bad)
    _, bad_blobs = S.unmarshal_blob_tx(bad)
    eng = RecordingCommitments()
    pre = P.precompute_commitments(txs, ctx=eng)
    assert pre[3] is None and eng.calls == 1
    assert all(bytes(b["ns"]) not in eng.batches[0] for b in bad_blobs) or which == "zero"
    n_good_blobs = sum(len(S.unmarshal_blob_tx(t)[1]) for i, t in enumerate(txs)
                       if i != 3 and S.unmarshal_blob_tx(t) is not None)
    assert len(eng.batches[0]) == n_good_blobs
    assert P.process_proposal_blob_txs(txs, ctx=RecordingCommitments()) == (3, code)


def test_namespace_rules():
    assert P.namespace_error(bytes(29)) == "ErrReservedNamespace"
    assert P.namespace_error(bytes(28) + b"\xff") == "ErrReservedNamespace"
    assert P.namespace_error(b"\xff" * 29) == "ErrReservedNamespace"
    assert P.namespace_error(bytes(19) + b"\x01" + bytes(9)) is None
    assert P.namespace_error(b"\x00" + b"\x01" + bytes(27)) == "ErrInvalidNamespace"  # version-0 prefix rule
    assert P.namespace_error(b"\x01" + bytes(28)) == "ErrInvalidNamespaceVersion"
    assert P.namespace_error(bytes(28)) == "ErrInvalidNamespace"


@pytest.mark.gpu
def test_gpu_proposal_prepass_one_call(ctx):
    """The product path: every commitment of a proposal (mainnet block 408's txs + synthetic BlobTxs) from ONE
    cda_blob_commitments call, equal to the oracle's; a tampered commitment is rejected at its index."""
    calls = []
    orig = ctx.blob_commitments

    def counted(*a, **kw):
        calls.append(len(a[1]))
        return orig(*a, **kw)

    ctx.blob_commitments = counted
    try:
        txs = mainnet_txs() + random_proposal(7, n_blob_txs=12)
        pre = P.precompute_commitments(txs, ctx=ctx)
        assert len(calls) == 1
        ref = OracleCommitments()
        for t, p in zip(txs, pre):
            b = S.unmarshal_blob_tx(t)
            if b is None:
                continue
            assert p == ref.blob_commitments([x["ns"] for x in b[1]], [x["data"] for x in b[1]])
        calls.clear()
        assert P.process_proposal_blob_txs(txs, ctx=ctx) == (None, None)
        assert len(calls) == 1
        bad, code = _tamper(9, "commitment")
        txs.insert(100, bad)
        assert P.process_proposal_blob_txs(txs, ctx=ctx) == (100, code)
    finally:
        ctx.blob_commitments = orig
