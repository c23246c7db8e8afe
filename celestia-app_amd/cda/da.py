"""pkg/da mirror (pkg/da/data_availability_header.go, celestia-app @ 2025-02-13)."""
import math

import numpy as np

from . import _native as N
from . import appconsts
from .rsmt2d import ExtendedDataSquare, LeoRSCodec

MAX_EXTENDED_SQUARE_WIDTH = appconsts.DEFAULT_SQUARE_SIZE_UPPER_BOUND * 2
MIN_EXTENDED_SQUARE_WIDTH = appconsts.MIN_SQUARE_SIZE * 2


class DAError(Exception):
    pass


def round_up_power_of_two(x):
    r = 1
    while r < x:
        r <<= 1
    return r


def square_size(n):
    """SquareSize(len) = RoundUpPowerOfTwo(ceil(sqrt(len)))  (:205-207)."""
    return round_up_power_of_two(int(math.ceil(math.sqrt(n))))


def is_power_of_two(n):
    return n > 0 and (n & (n - 1)) == 0


def extend_shares(shares, codec=None):
    """ExtendShares (:65-75).  As go/cda's ExtendSharesOn: a square of 512-byte shares is written straight into Q0 of
    the EDS buffer and extended in place (cda_extend_commit_eds); anything else goes through cda_extend_commit, which
    raises the reference's errors in its order (not a square, chunk size)."""
    if not is_power_of_two(len(shares)):
        raise DAError(f"number of shares is not a power of 2: got {len(shares)}")
    codec = codec or LeoRSCodec()
    k = square_size(len(shares))
    if k * k == len(shares) and all(len(s) == appconsts.SHARE_SIZE for s in shares):
        eds = np.empty((4 * k * k, appconsts.SHARE_SIZE), np.uint8)
        q0 = eds.reshape(2 * k, 2 * k, appconsts.SHARE_SIZE)[:k, :k]
        for i, s in enumerate(shares):
            q0[i // k, i % k] = np.frombuffer(bytes(s), np.uint8)
        rr, cr, _ = codec.ctx.extend_commit_eds(eds)
        return ExtendedDataSquare(eds, 2 * k, k, codec, rr, cr)
    arr = np.stack([np.frombuffer(bytes(s), np.uint8) for s in shares])
    eds, rr, cr, _ = codec.ctx.extend_commit(arr)
    k = int(round(len(shares) ** 0.5))
    return ExtendedDataSquare(eds, 2 * k, k, codec, rr, cr)


def new_data_availability_header_from_shares(shares, ctx=None):
    """NewDataAvailabilityHeaderFromShares (go/patches/0004: PrepareProposal / ProcessProposal read only the header,
    app/prepare_proposal.go:65-93, app/process_proposal.go:137-151) = NewDataAvailabilityHeader(ExtendShares(s)) with
    the same roots, hash and errors, from one cda_extend_commit that copies no EDS back."""
    if not is_power_of_two(len(shares)):
        raise DAError(f"number of shares is not a power of 2: got {len(shares)}")
    ctx = ctx or N.default_context()
    arr = np.stack([np.frombuffer(bytes(s), np.uint8) for s in shares])
    _, rr, cr, h = ctx.extend_commit(arr, want_eds=False)
    dah = DataAvailabilityHeader(list(rr), list(cr), ctx=ctx)
    dah._hash = h
    return dah


class DataAvailabilityHeader:
    def __init__(self, row_roots=None, column_roots=None, ctx=None):
        self.row_roots = [bytes(r) for r in (row_roots or [])]
        self.column_roots = [bytes(r) for r in (column_roots or [])]
        self._hash = b""
        self._ctx = ctx

    def hash(self):
        """Hash (:92-108): RFC-6962 root of rowRoots ‖ columnRoots (memoised)."""
        if self._hash:
            return self._hash
        ctx = self._ctx or N.default_context()
        n = len(self.row_roots)
        if n == 0 and len(self.column_roots) == 0:
            self._hash = ctx.dah_hash(None, None)
        else:
            self._hash = ctx.dah_hash(np.frombuffer(b"".join(self.row_roots), np.uint8).reshape(n, -1),
                                      np.frombuffer(b"".join(self.column_roots), np.uint8).reshape(n, -1))
        return self._hash

    def string(self):
        return self.hash().hex().upper()

    def equals(self, other):
        return self.hash() == other.hash()

    def is_zero(self):
        return len(self.column_roots) == 0 or len(self.row_roots) == 0

    def square_size(self):
        return len(self.row_roots) // 2

    def validate_basic(self):
        """ValidateBasic (:134-162)."""
        if len(self.column_roots) < MIN_EXTENDED_SQUARE_WIDTH or len(self.row_roots) < MIN_EXTENDED_SQUARE_WIDTH:
            raise DAError(f"minimum valid DataAvailabilityHeader has at least {MIN_EXTENDED_SQUARE_WIDTH} "
                          "row and column roots")
        if len(self.column_roots) > MAX_EXTENDED_SQUARE_WIDTH or len(self.row_roots) > MAX_EXTENDED_SQUARE_WIDTH:
            raise DAError(f"maximum valid DataAvailabilityHeader has at most {MAX_EXTENDED_SQUARE_WIDTH} "
                          "row and column roots")
        if len(self.column_roots) != len(self.row_roots):
            raise DAError(f"unequal number of row and column roots: row {len(self.row_roots)} "
                          f"col {len(self.column_roots)}")
        if len(self.hash()) != appconsts.HASH_LENGTH:
            raise DAError("wrong hash: expected size to be 32 bytes")


    def to_proto(self):
        """ToProto (:110-119) in wire form: celestia.core.v1.da.DataAvailabilityHeader
        {repeated bytes row_roots = 1; repeated bytes column_roots = 2}
        (proto/celestia/core/v1/da/data_availability_header.proto:16-21)."""
        out = bytearray()
        for r in self.row_roots:
            out += b"\x0a" + _varint(len(r)) + r
        for c in self.column_roots:
            out += b"\x12" + _varint(len(c)) + c
        return bytes(out)


def _varint(v):
    out = bytearray()
    while True:
        b, v = v & 0x7F, v >> 7
        out.append(b | 0x80 if v else b)
        if not v:
            return bytes(out)


def _read_varint(buf, i):
    shift = v = 0
    while True:
        if i >= len(buf):
            raise DAError("truncated varint")
        b = buf[i]
        i += 1
        v |= (b & 0x7F) << shift
        shift += 7
        if not b & 0x80:
            return v, i


def data_availability_header_from_proto(buf, ctx=None):
    """DataAvailabilityHeaderFromProto (:121-131): decode the wire message, then ValidateBasic."""
    buf = bytes(buf)
    rows, cols, i = [], [], 0
    while i < len(buf):
        key, i = _read_varint(buf, i)
        if key & 7 != 2:
            raise DAError(f"unexpected wire type {key & 7}")
        n, i = _read_varint(buf, i)
        if i + n > len(buf):
            raise DAError("truncated DataAvailabilityHeader")
        if key >> 3 == 1:
            rows.append(buf[i:i + n])
        elif key >> 3 == 2:
            cols.append(buf[i:i + n])
        i += n
    dah = DataAvailabilityHeader(rows, cols, ctx=ctx)
    dah.validate_basic()
    return dah


def new_data_availability_header(eds: ExtendedDataSquare):
    """NewDataAvailabilityHeader (:44-63)."""
    dah = DataAvailabilityHeader(eds.row_roots(), eds.col_roots(), ctx=eds.codec.ctx)
    dah.hash()
    return dah


def tail_padding_share():
    """go-square shares.TailPaddingShare: ns ‖ info(0x01) ‖ seqlen 0 ‖ zeros (specs shares.md:71-81)."""
    s = bytearray(appconsts.SHARE_SIZE)
    s[:29] = appconsts.TAIL_PADDING_NAMESPACE
    s[29] = 0x01
    return bytes(s)


def min_shares():
    return [tail_padding_share()]


def min_data_availability_header():
    """MinDataAvailabilityHeader (:179-190)."""
    return new_data_availability_header(extend_shares(min_shares()))
