"""ProcessProposal's BlobTx checks with every share commitment of the proposal from ONE batched GPU call.

Reference: app/process_proposal.go:56-118 walks req.BlockData.Txs and runs blobtypes.ValidateBlobTx on each BlobTx
(:106); ValidateBlobTx ends by recomputing every blob's share commitment with go-square
inclusion.CreateCommitment and comparing it with the MsgPayForBlobs' (x/blob/types/blob_tx.go:97-105).  The
engine's form (go/patches/0003): a pre-pass collects the blobs of every BlobTx and computes all of their
commitments in one cda_blob_commitments call, then the loop runs the same checks in the same order and compares
against the precomputed values.  Only blobs that ValidateBlobs would accept (29-byte namespace, non-empty data,
supported share version) enter the batch, so the batched call cannot fail on a bad blob; a tx whose blobs do not
all qualify gets no precomputed values and fails (or passes) exactly where the reference's checks put it.

The mirror parses the wire format itself (TxRaw -> TxBody -> Any -> MsgPayForBlobs, proto/celestia/blob/v1/
tx.proto:17-34).  It does not decode the rest of an sdk.Tx, check the signer's bech32 address
(payforblob.go:136) or run the ante handler: those are host-side checks outside the DA path.
"""
from . import appconsts
from . import _native as N
from .square import parse_fields, read_varint, unmarshal_blob_tx

PFB_URL = b"/celestia.blob.v1.MsgPayForBlobs"
NAMESPACE_VERSION_ZERO_PREFIX = 18
MAX_PRIMARY_RESERVED = bytes(28) + b"\xff"            # specs/src/specs/namespace.md:81
MIN_SECONDARY_RESERVED = b"\xff" * 28 + b"\x00"       # namespace.md:82
SUPPORTED_BLOB_NAMESPACE_VERSIONS = (0,)


class BlobTxError(Exception):
    """A ValidateBlobTx failure; `code` names the reference's error (x/blob/types/errors.go)."""

    def __init__(self, code, detail=""):
        self.code = code
        super().__init__(f"{code}{': ' + detail if detail else ''}")


def _uvarints(fields, num):
    out = []
    for f, wt, v in fields:
        if f != num:
            continue
        if wt == 0:
            out.append(v)
        elif wt == 2:
            i = 0
            while i < len(v):
                x, i = read_varint(v, i)
                out.append(x)
    return out


def decode_pfb_tx(tx):
    """sdk TxRaw{body_bytes = 1} -> TxBody{messages = 1} -> the messages as (type_url, value) pairs."""
    raw = parse_fields(tx)
    if raw is None:
        raise BlobTxError("ErrTxDecode")
    body = next((v for f, wt, v in raw if f == 1 and wt == 2), None)
    fields = parse_fields(body) if body is not None else None
    if fields is None:
        raise BlobTxError("ErrTxDecode")
    msgs = []
    for f, wt, v in fields:
        if f == 1 and wt == 2:
            a = parse_fields(v)
            if a is None:
                raise BlobTxError("ErrTxDecode")
            url = next((x for g, t, x in a if g == 1 and t == 2), b"")
            val = next((x for g, t, x in a if g == 2 and t == 2), b"")
            msgs.append((url, val))
    return msgs


def parse_pfb(value):
    m = parse_fields(value)
    if m is None:
        raise BlobTxError("ErrTxDecode")
    return {"signer": next((v for f, wt, v in m if f == 1 and wt == 2), b""),
            "namespaces": [v for f, wt, v in m if f == 2 and wt == 2],
            "blob_sizes": _uvarints(m, 3),
            "share_commitments": [v for f, wt, v in m if f == 4 and wt == 2],
            "share_versions": _uvarints(m, 8)}


def namespace_error(ns):
    """appns.From / appns.New + ValidateBlobNamespace (payforblob.go:184-194) -> error code or None."""
    if len(ns) != appconsts.NAMESPACE_SIZE:
        return "ErrInvalidNamespace"
    version, nid = ns[0], ns[1:]
    if version == 0 and any(nid[:NAMESPACE_VERSION_ZERO_PREFIX]):
        return "ErrInvalidNamespace"  # version 0 ids carry 18 leading zero bytes (namespace.md:35)
    if ns <= MAX_PRIMARY_RESERVED or ns >= MIN_SECONDARY_RESERVED:
        return "ErrReservedNamespace"
    if version not in SUPPORTED_BLOB_NAMESPACE_VERSIONS:
        return "ErrInvalidNamespaceVersion"
    return None


def validate_basic(pfb):
    """MsgPayForBlobs.ValidateBasic (payforblob.go:96-147), signer address excepted."""
    for key, code in (("namespaces", "ErrNoNamespaces"), ("share_versions", "ErrNoShareVersions"),
                      ("blob_sizes", "ErrNoBlobSizes"), ("share_commitments", "ErrNoShareCommitments")):
        if not pfb[key]:
            raise BlobTxError(code)
    n = len(pfb["namespaces"])
    if not (n == len(pfb["share_versions"]) == len(pfb["blob_sizes"]) == len(pfb["share_commitments"])):
        raise BlobTxError("ErrMismatchedNumberOfPFBComponent")
    for ns in pfb["namespaces"]:
        e = namespace_error(ns)
        if e:
            raise BlobTxError(e)
    if any(v != appconsts.SHARE_VERSION_ZERO for v in pfb["share_versions"]):
        raise BlobTxError("ErrUnsupportedShareVersion")
    if any(len(c) != appconsts.HASH_LENGTH for c in pfb["share_commitments"]):
        raise BlobTxError("ErrInvalidShareCommitment")


def validate_blobs(blobs):
    """ValidateBlobs (payforblob.go:213-240)."""
    if not blobs:
        raise BlobTxError("ErrNoBlobs")
    for b in blobs:
        e = namespace_error(b["ns"])
        if e:
            raise BlobTxError(e)
        if not b["data"]:
            raise BlobTxError("ErrZeroBlobSize")
        if b["share_version"] not in appconsts.SUPPORTED_SHARE_VERSIONS:
            raise BlobTxError("ErrUnsupportedShareVersion")


def _batchable(blobs):
    """A BlobTx's blobs enter the batched commitment call exactly when ValidateBlobs accepts them (the filter of the
    Go patch's PrecomputeCommitments: reserved namespaces, namespace version and the v0 prefix included)."""
    try:
        validate_blobs(blobs)
    except BlobTxError:
        return False
    return True


def precompute_commitments(txs, subtree_root_threshold=appconsts.SUBTREE_ROOT_THRESHOLD, ctx=None):
    """The pre-pass: every BlobTx's commitments in ONE cda_blob_commitments call.  -> list (one entry per tx): the
    tx's commitments, or None for a normal tx / a BlobTx with a blob ValidateBlobs would reject / every tx when the
    batch call fails (go/patches/0003 PrecomputeCommitments: the per-tx checks then compute their own)."""
    parsed = [unmarshal_blob_tx(t) for t in txs]
    take = [i for i, p in enumerate(parsed) if p is not None and _batchable(p[1])]
    out = [None] * len(txs)
    if not take:
        return out
    blobs = [b for i in take for b in parsed[i][1]]
    ctx = ctx or N.default_context()
    try:
        got = ctx.blob_commitments([b["ns"] for b in blobs], [b["data"] for b in blobs],
                                   [b["share_version"] for b in blobs], subtree_root_threshold)
    except N.CdaError:
        return out  # as the Go pre-pass: a failed batch leaves every tx to compute its own commitments
    if len(got) != len(blobs):
        return out
    pos = 0
    for i in take:
        n = len(parsed[i][1])
        out[i] = got[pos:pos + n]
        pos += n
    return out


def validate_blob_tx(raw_tx, subtree_root_threshold=appconsts.SUBTREE_ROOT_THRESHOLD, precomputed=None, ctx=None):
    """ValidateBlobTx (x/blob/types/blob_tx.go:37-107) on one BlobTx; raises BlobTxError.  `precomputed`: this tx's
    commitments from precompute_commitments (None: computed here, one call for this tx's blobs)."""
    p = unmarshal_blob_tx(raw_tx)
    if p is None:
        raise BlobTxError("ErrNoBlobs")
    tx, blobs = p
    msgs = decode_pfb_tx(tx)
    if len(msgs) != 1:
        raise BlobTxError("ErrMultipleMsgsInBlobTx")
    url, value = msgs[0]
    if url != PFB_URL:
        raise BlobTxError("ErrNoPFB")
    pfb = parse_pfb(value)
    validate_basic(pfb)
    validate_blobs(blobs)
    if [len(b["data"]) for b in blobs] != pfb["blob_sizes"]:
        raise BlobTxError("ErrBlobSizeMismatch")
    for i, ns in enumerate(pfb["namespaces"]):
        if blobs[i]["ns"] != ns:
            raise BlobTxError("ErrNamespaceMismatch")
    if precomputed is None or len(precomputed) != len(blobs):
        ctx = ctx or N.default_context()
        precomputed = ctx.blob_commitments([b["ns"] for b in blobs], [b["data"] for b in blobs],
                                           [b["share_version"] for b in blobs], subtree_root_threshold)
    for i, c in enumerate(pfb["share_commitments"]):
        if precomputed[i] != c:
            raise BlobTxError("ErrInvalidShareCommitment")


def process_proposal_blob_txs(txs, subtree_root_threshold=appconsts.SUBTREE_ROOT_THRESHOLD, ctx=None):
    """The BlobTx part of ProcessProposal's loop (process_proposal.go:56-118) with the batched pre-pass.
    -> (None, None) if every BlobTx is valid, else (index of the first invalid tx, its error code)."""
    pre = precompute_commitments(txs, subtree_root_threshold, ctx)
    for idx, raw in enumerate(txs):
        if unmarshal_blob_tx(raw) is None:
            continue  # normal txs: decoding / ante checks, outside the DA path
        try:
            validate_blob_tx(raw, subtree_root_threshold, pre[idx], ctx)
        except BlobTxError as e:
            return idx, e.code
    return None, None
