"""go-square square construction mirror: transactions -> original data square (ODS).

The step before the DA path: app/prepare_proposal.go:54 and
app/process_proposal.go:121 call go-square v1.0.1 square.Construct / Build and
shares.ToBytes (go.mod:9, not vendored), then da.ExtendShares. The rules are
restated from the reference's specs and call sites:

  * txs split into normal txs and BlobTxs (blob.UnmarshalBlobTx: BlobTx{tx=1,
    blobs=2, type_id=3 "BLOB"}); blobs sorted stably by namespace, PFB priority
    order kept within a namespace (test/util/malicious/out_of_order_builder.go:24-150
    is the builder and its Export, here without the malicious swap);
  * compact shares for the TRANSACTION and PAY_FOR_BLOB namespaces: varint-delimited
    units, sequence length and reserved bytes (specs/src/specs/shares.md:61-80);
    PFBs are wrapped in IndexWrapper{tx=1, share_indexes=2, type_id=3 "INDX"};
  * sparse blob shares, namespace / reserved / tail padding (shares.md:31-122);
  * every blob starts at a multiple of its SubTreeWidth
    (specs/src/specs/data_square_layout.md:47-60);
  * the PFB share reservation assumes worst-case share indexes of
    SquareSizeUpperBound^2 (pkg/appconsts/v1/app_consts.go:5).

Pinned on real data: mainnet block 408's txs (the reference's fixture
x/blob/test/testdata/block_response.json) construct the square whose DAH is the
block header's data_hash (tests/test_square.py). Host logic only: the bytes are
layout, not arithmetic; the extension and hashing run in libcda.
"""
import math

from . import appconsts
from .inclusion import next_share_index, sparse_shares_needed, sub_tree_width

SHARE = appconsts.SHARE_SIZE
NS = appconsts.NAMESPACE_SIZE
TX_NAMESPACE = bytes(28) + b"\x01"
PAY_FOR_BLOB_NAMESPACE = bytes(28) + b"\x04"
PRIMARY_RESERVED_PADDING_NAMESPACE = bytes(28) + b"\xff"
TAIL_PADDING_NAMESPACE = appconsts.TAIL_PADDING_NAMESPACE
FIRST_COMPACT_SHARE_CONTENT_SIZE = SHARE - NS - 1 - 4 - 4  # 474
CONTINUATION_COMPACT_SHARE_CONTENT_SIZE = SHARE - NS - 1 - 4  # 478


class SquareError(Exception):
    pass


# ---- protobuf wire format --------------------------------------------------------------------
def varint(v):
    out = bytearray()
    while True:
        b, v = v & 0x7F, v >> 7
        out.append(b | 0x80 if v else b)
        if not v:
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
    """-> list of (field, wire type, value), or None if `buf` is not a well-formed message."""
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
    """blob.UnmarshalBlobTx -> (tx, [{"ns", "data", "share_version"}]) or None for a normal tx."""
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
        for f, wt, v in parse_fields(b) or []:
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


def marshal_index_wrapper(tx, share_indexes):
    """blob.MarshalIndexWrapper: IndexWrapper{tx=1, share_indexes=2 (packed), type_id=3 "INDX"}."""
    out = b"\x0a" + varint(len(tx)) + tx
    if share_indexes:
        packed = b"".join(varint(x) for x in share_indexes)
        out += b"\x12" + varint(len(packed)) + packed
    return out + b"\x1a" + varint(4) + b"INDX"


# ---- shares ------------------------------------------------------------------------------------
def compact_shares_needed(sequence_len):
    if sequence_len == 0:
        return 0
    if sequence_len <= FIRST_COMPACT_SHARE_CONTENT_SIZE:
        return 1
    return 1 + math.ceil((sequence_len - FIRST_COMPACT_SHARE_CONTENT_SIZE) / CONTINUATION_COMPACT_SHARE_CONTENT_SIZE)


def compact_layout(units):
    """The varint-delimited sequence of `units` and, per compact share, its reserved bytes value: the offset in
    the share of the first unit that starts in it, 0 if none (shares.md:61-80)."""
    seq = b"".join(varint(len(u)) + u for u in units)
    starts, off = [], 0
    for u in units:
        starts.append(off)
        off += len(varint(len(u))) + len(u)
    reserved, pos = [], 0
    for s in range(compact_shares_needed(len(seq))):
        first = s == 0
        cap = FIRST_COMPACT_SHARE_CONTENT_SIZE if first else CONTINUATION_COMPACT_SHARE_CONTENT_SIZE
        data_start = NS + 1 + (4 if first else 0) + 4
        lo, hi = pos, pos + cap
        first_unit = next((st for st in starts if lo <= st < hi), None)
        reserved.append(0 if first_unit is None else data_start + (first_unit - lo))
        pos = hi
    return seq, reserved


def compact_shares(ns, units):
    """CompactShareSplitter: varint-delimited units, sequence length, reserved bytes (shares.md:61-80)."""
    seq, reserved = compact_layout(units)
    out, pos = [], 0
    for s, resv in enumerate(reserved):
        first = s == 0
        header = ns + bytes([1 if first else 0]) + (len(seq).to_bytes(4, "big") if first else b"")
        cap = FIRST_COMPACT_SHARE_CONTENT_SIZE if first else CONTINUATION_COMPACT_SHARE_CONTENT_SIZE
        share = header + resv.to_bytes(4, "big") + seq[pos:pos + cap]
        out.append(share + bytes(SHARE - len(share)))
        pos += cap
    return out


def sparse_shares(ns, data, share_version=appconsts.SHARE_VERSION_ZERO):
    """SparseShareSplitter.Write: ns ‖ info ‖ [sequence length] ‖ data ‖ zeros (shares.md:31-60)."""
    out, pos = [], 0
    for s in range(sparse_shares_needed(len(data))):
        first = s == 0
        header = ns + bytes([(share_version << 1) | (1 if first else 0)])
        if first:
            header += len(data).to_bytes(4, "big")
        share = header + data[pos:pos + SHARE - len(header)]
        out.append(share + bytes(SHARE - len(share)))
        pos += SHARE - len(header)
    return out


def padding_share(ns):
    """Namespace / reserved / tail padding share: ns ‖ info(first) ‖ sequence length 0 ‖ zeros (shares.md:82-122)."""
    share = ns + b"\x01" + bytes(4)
    return share + bytes(SHARE - len(share))


# ---- square.Construct ----------------------------------------------------------------------------
def plan(txs, max_square_size=appconsts.DEFAULT_SQUARE_SIZE_UPPER_BOUND,
         subtree_root_threshold=appconsts.SUBTREE_ROOT_THRESHOLD, square_size_upper_bound=None):
    """square.Construct's layout (go-square v1.0.1) without the share bytes: (k, segments, info).  A segment is
    a run of shares of one sequence: compact (TRANSACTION / PAY_FOR_BLOB units), sparse (one blob) or padding;
    render() turns them into shares on the host, cda_construct_extend_commit on the device."""
    upper = square_size_upper_bound or max_square_size
    normal, pfbs, blobs = [], [], []
    for raw in txs:
        bt = unmarshal_blob_tx(raw)
        if bt is None:
            normal.append(raw)
            continue
        tx, bl = bt
        pfbs.append({"tx": tx, "idx": [0] * len(bl)})
        for j, b in enumerate(bl):
            n = sparse_shares_needed(len(b["data"]))
            blobs.append({"blob": b, "pfb": len(pfbs) - 1, "j": j, "n": n,
                          "max_pad": sub_tree_width(n, subtree_root_threshold) - 1})
    tx_seq = sum(len(varint(len(t))) + len(t) for t in normal)
    worst = upper * upper
    pfb_seq = sum(len(varint(len(w))) + len(w)
                  for w in (marshal_index_wrapper(p["tx"], [worst] * len(p["idx"])) for p in pfbs))
    tx_shares, pfb_reserved = compact_shares_needed(tx_seq), compact_shares_needed(pfb_seq)
    current = tx_shares + pfb_reserved + sum(b["n"] + b["max_pad"] for b in blobs)
    ss = 1
    while ss * ss < max(current, 1):
        ss <<= 1
    if ss > max_square_size:
        raise SquareError(f"square size {ss} exceeds the maximum {max_square_size}")
    blobs.sort(key=lambda b: b["blob"]["ns"])  # stable: PFB order within a namespace
    non_reserved_start = tx_shares + pfb_reserved
    cursor = end_last = non_reserved_start
    for i, b in enumerate(blobs):
        cursor = next_share_index(cursor, b["n"], subtree_root_threshold)
        if i == 0:
            non_reserved_start = cursor
        pad = cursor - end_last
        if pad > b["max_pad"]:
            raise SquareError("blob padding exceeds its subtree width")
        pfbs[b["pfb"]]["idx"][b["j"]] = cursor
        b["start"] = cursor
        cursor += b["n"]
        end_last = cursor
    pfb_units = [marshal_index_wrapper(p["tx"], p["idx"]) for p in pfbs]
    if compact_shares_needed(sum(len(varint(len(u))) + len(u) for u in pfb_units)) > pfb_reserved:
        raise SquareError("PFB shares exceed their reservation")
    # the square as segments (row-major share runs): compact txs, compact PFBs, reserved padding up to the
    # first blob, blobs with namespace padding between them, tail padding
    segs, n = [], 0

    def add(kind, count, ns, payload=None):
        nonlocal n
        if count > 0:
            segs.append({"kind": kind, "first": n, "n": count, "ns": ns, "payload": payload})
            n += count
    add("compact", tx_shares, TX_NAMESPACE, normal)
    add("compact", compact_shares_needed(sum(len(varint(len(u))) + len(u) for u in pfb_units)),
        PAY_FOR_BLOB_NAMESPACE, pfb_units)
    pfb_count = n - tx_shares
    if blobs:
        add("padding", non_reserved_start - n, PRIMARY_RESERVED_PADDING_NAMESPACE)
        prev_end = None
        for b in blobs:
            start = b["start"]
            if prev_end is not None:
                add("padding", start - prev_end, prev_ns)
            add("sparse", b["n"], b["blob"]["ns"], b["blob"])
            prev_end, prev_ns = start + b["n"], b["blob"]["ns"]
    add("padding", ss * ss - n, TAIL_PADDING_NAMESPACE)
    info = {"normal_txs": len(normal), "pfbs": len(pfbs), "blobs": len(blobs), "tx_shares": tx_shares,
            "pfb_shares": pfb_count, "pfb_reserved": pfb_reserved,
            "first_blob": non_reserved_start if blobs else None, "current_size": current,
            "pfb_share_indexes": [p["idx"] for p in pfbs]}
    return ss, segs, info


def render(segs):
    """Host bytes of a plan (shares.ToBytes order): list of 512-byte shares."""
    out = []
    for sg in segs:
        if sg["kind"] == "compact":
            out += compact_shares(sg["ns"], sg["payload"])
        elif sg["kind"] == "sparse":
            out += sparse_shares(sg["ns"], sg["payload"]["data"], sg["payload"]["share_version"])
        else:
            out += [padding_share(sg["ns"])] * sg["n"]
    return out


def construct(txs, max_square_size=appconsts.DEFAULT_SQUARE_SIZE_UPPER_BOUND,
              subtree_root_threshold=appconsts.SUBTREE_ROOT_THRESHOLD, square_size_upper_bound=None):
    """square.Construct(txs, maxSquareSize, subtreeRootThreshold) -> (square size k, k*k shares, layout info).

    square_size_upper_bound sizes the PFB share-index reservation (defaults to max_square_size).
    """
    ss, segs, info = plan(txs, max_square_size, subtree_root_threshold, square_size_upper_bound)
    return ss, render(segs), info


SEG_KIND = {"compact": 0, "sparse": 1, "padding": 2}  # CDA_SEG_* (include/cda.h)


def device_plan(segs):
    """The plan as cda_share_segment records + payload bytes + compact reserved offsets (numpy arrays)."""
    import numpy as np
    from ._native import ShareSegment
    recs = (ShareSegment * len(segs))()
    data, reserved, off = [], [], 0
    for i, sg in enumerate(segs):
        r = recs[i]
        r.kind, r.first_share, r.nshares, r.share_version = SEG_KIND[sg["kind"]], sg["first"], sg["n"], 0
        r.ns[:] = list(sg["ns"])
        if sg["kind"] == "compact":
            seq, resv = compact_layout(sg["payload"])
            r.reserved_off = len(reserved)
            reserved += resv
            payload = seq
        elif sg["kind"] == "sparse":
            payload = sg["payload"]["data"]
            r.share_version = sg["payload"]["share_version"]
        else:
            payload = b""
        r.data_off, r.data_len = off, len(payload)
        data.append(payload)
        off += len(payload)
    return recs, np.frombuffer(b"".join(data) or b"\0", np.uint8), np.array(reserved or [0], np.uint32)


def segments_from_shares(shares):
    """The layout plan read back from a constructed square's shares (go/cda/square.go SegmentsFromShares, its Go
    twin): ns ‖ info (share version << 1 | sequence start) ‖ sequence length (first share) ‖ reserved bytes (compact
    shares) ‖ payload.  A run of identical shares of sequence length 0 outside the compact namespaces is padding.
    Returns device_plan's triple (cda_share_segment records, payload bytes, reserved values), so only the payload
    crosses PCIe in cda_construct_extend_commit."""
    import numpy as np
    from ._native import ShareSegment
    segs, data, reserved, off, i = [], [], [], 0, 0
    while i < len(shares):
        sh = bytes(shares[i])
        if len(sh) != SHARE:
            raise SquareError(f"share {i} is {len(sh)} bytes")
        ns, info = sh[:NS], sh[NS]
        if not info & 1:
            raise SquareError(f"share {i} continues no sequence")
        seq_len = int.from_bytes(sh[NS + 1:NS + 5], "big")
        compact = ns in (TX_NAMESPACE, PAY_FOR_BLOB_NAMESPACE)
        if not compact and seq_len == 0:
            j = i + 1
            while j < len(shares) and bytes(shares[j]) == sh:
                j += 1
            segs.append(dict(kind=SEG_KIND["padding"], first=i, n=j - i, version=info >> 1, ns=ns, off=off, len=0,
                             roff=0))
            i = j
            continue
        hdr0, hdrn = (NS + 9, NS + 5) if compact else (NS + 5, NS + 1)
        payload, resv, j = bytearray(), [], i
        while j < len(shares) and (j == i or (bytes(shares[j][:NS]) == ns and not shares[j][NS] & 1)):
            h = hdr0 if j == i else hdrn
            if compact:
                resv.append(int.from_bytes(bytes(shares[j][h - 4:h]), "big"))
            payload += bytes(shares[j][h:])
            j += 1
        if len(payload) < seq_len:
            raise SquareError(f"sequence at share {i} is shorter than its length {seq_len}")
        segs.append(dict(kind=SEG_KIND["compact" if compact else "sparse"], first=i, n=j - i, version=info >> 1,
                         ns=ns, off=off, len=seq_len, roff=len(reserved) if compact else 0))
        data.append(bytes(payload[:seq_len]))
        reserved += resv
        off += seq_len
        i = j
    recs = (ShareSegment * len(segs))()
    for r, sg in zip(recs, segs):
        r.kind, r.first_share, r.nshares, r.share_version = sg["kind"], sg["first"], sg["n"], sg["version"]
        r.data_off, r.data_len, r.reserved_off = sg["off"], sg["len"], sg["roff"]
        r.ns[:] = list(sg["ns"])
    return recs, np.frombuffer(b"".join(data) or b"\0", np.uint8), np.array(reserved or [0], np.uint32)
