"""rsmt2d-shaped API (github.com/celestiaorg/rsmt2d v0.12.0, go.mod:13) over libcda.

Mirrors the pieces celestia-app uses: the Codec interface (LeoRSCodec,
selected at pkg/appconsts/global_consts.go:92), ComputeExtendedDataSquare,
ExtendedDataSquare.{RowRoots,ColRoots,Row,Col,GetCell,SetCell,Flattened,Width},
Repair and its error types.  All arithmetic runs in libcda on the GPU.
"""
import numpy as np

from . import _native as N

ROW = N.AXIS_ROW
COL = N.AXIS_COL
LEOPARD = "Leopard"


class ErrUnrepairableDataSquare(Exception):
    """rsmt2d.ErrUnrepairableDataSquare"""


class ErrByzantineData(Exception):
    """rsmt2d.ErrByzantineData{Axis, Index, Shares}"""

    def __init__(self, axis, index, shares=None):
        self.axis, self.index, self.shares = axis, index, shares
        super().__init__(f"byzantine {'row' if axis == ROW else 'col'}: {index}")


class LeoRSCodec:
    """rsmt2d.LeoRSCodec: Leopard RS, GF(2^8) for 2k <= 256 else GF(2^16)."""

    def __init__(self, ctx=None):
        self._ctx = ctx

    @property
    def ctx(self):
        return self._ctx or N.default_context()

    def encode(self, data):
        """Codec.Encode(data [][]byte) ([][]byte, error): k data shards -> k parity shards."""
        arr = np.stack([np.frombuffer(bytes(d), np.uint8) for d in data])
        par = self.ctx.rs_encode(arr)
        return [bytes(p) for p in par]

    def decode(self, shards):
        """Codec.Decode: shards with None for missing -> all shards."""
        n = len(shards)
        L = max(len(s) for s in shards if s is not None)
        arr = np.zeros((n, L), np.uint8)
        present = np.zeros(n, np.uint8)
        for i, s in enumerate(shards):
            if s is not None:
                arr[i] = np.frombuffer(bytes(s), np.uint8)
                present[i] = 1
        out = self.ctx.rs_decode(arr, present)
        return [bytes(r) for r in out]

    def max_chunks(self):
        return int(N.lib().cda_rs_max_chunks())

    def name(self):
        return N.lib().cda_rs_name().decode()

    def validate_chunk_size(self, chunk_size):
        rc = N.lib().cda_rs_validate_chunk_size(int(chunk_size))
        if rc:
            raise N.CdaError(rc, f"chunkSize {chunk_size} must be a multiple of 64 bytes")


def new_leo_rs_codec(ctx=None):
    return LeoRSCodec(ctx)


class ExtendedDataSquare:
    """rsmt2d.ExtendedDataSquare backed by a (width*width, 512) array."""

    def __init__(self, cells, width, original_width, codec=None, row_roots=None, col_roots=None, present=None):
        self.cells = cells
        self._width = width
        self.original_data_width = original_width
        self.codec = codec or LeoRSCodec()
        self._row_roots = row_roots
        self._col_roots = col_roots
        self.present = present if present is not None else np.ones(width * width, np.uint8)

    def width(self):
        return self._width

    def get_cell(self, r, c):
        if not self.present[r * self._width + c]:
            return None
        return bytes(self.cells[r * self._width + c])

    def set_cell(self, r, c, data):
        if self.present[r * self._width + c]:
            raise ValueError(f"cannot set cell ({r}, {c}) as it already has a value")
        self.cells[r * self._width + c] = np.frombuffer(bytes(data), np.uint8)
        self.present[r * self._width + c] = 1
        self._row_roots = self._col_roots = None

    def row(self, i):
        return [self.get_cell(i, c) for c in range(self._width)]

    def col(self, i):
        return [self.get_cell(r, i) for r in range(self._width)]

    def flattened(self):
        return [self.get_cell(i // self._width, i % self._width) for i in range(self._width ** 2)]

    def _compute_roots(self):
        if not self.present.all():
            raise ValueError("can not compute roots of incomplete EDS")
        rr, cr, _ = self.codec.ctx.commit_eds(self.cells)
        self._row_roots, self._col_roots = rr, cr

    def row_roots(self):
        if self._row_roots is None:
            self._compute_roots()
        return [bytes(r) for r in self._row_roots]

    def col_roots(self):
        if self._col_roots is None:
            self._compute_roots()
        return [bytes(r) for r in self._col_roots]

    def repair(self, row_roots, col_roots):
        """(*ExtendedDataSquare).Repair(rowRoots, colRoots) — in place."""
        rr = np.stack([np.frombuffer(bytes(r), np.uint8) for r in row_roots])
        cr = np.stack([np.frombuffer(bytes(r), np.uint8) for r in col_roots])
        try:
            eds, pres = self.codec.ctx.repair(self.cells, self.present, rr, cr)
        except N.CdaError as e:
            if e.code == N.E_UNREPAIRABLE:
                raise ErrUnrepairableDataSquare() from e
            if e.code == N.E_BYZANTINE:
                raise ErrByzantineData(e.axis, e.index) from e
            raise
        self.cells[:] = eds
        self.present[:] = pres
        self._row_roots, self._col_roots = rr, cr


def compute_extended_data_square(data, codec=None, tree_constructor=None):
    """rsmt2d.ComputeExtendedDataSquare(data, codec, treeCreatorFn).

    The extension always runs on the device.  With no tree constructor, or wrapper.NewConstructor(k) (the one
    pkg/da passes, data_availability_header.go:74), the fused device path also computes every root.  Any other
    TreeConstructorFn (e.g. pkg/inclusion's EDSSubTreeRootCacher, nmt_caching.go:96-109) gets the reference's
    semantics: rsmt2d builds one tree per axis through it, pushes that axis's cells in order and takes Root()."""
    codec = codec or LeoRSCodec()
    if len(data) > codec.max_chunks():
        raise ValueError("number of chunks exceeds the maximum")
    arr = np.stack([np.frombuffer(bytes(d), np.uint8) for d in data]) if len(data) else np.zeros((0, 512), np.uint8)
    k = int(round(len(data) ** 0.5))
    fused = tree_constructor is None or getattr(tree_constructor, "cda_erasured_square_size", None) == k
    eds, rr, cr, _ = codec.ctx.extend_commit(arr)
    sq = ExtendedDataSquare(eds, 2 * k, k, codec, rr, cr)
    if not fused:
        sq._row_roots, sq._col_roots = _roots_through(sq, tree_constructor)
    return sq




def _roots_through(sq, tree_constructor):
    """rsmt2d computeRoots with a caller's TreeConstructorFn: rows then columns, each axis pushed in order."""
    roots = []
    for axis, cells in ((ROW, sq.row), (COL, sq.col)):
        out = []
        for i in range(sq._width):
            tree = tree_constructor(axis, i)
            for share in cells(i):
                tree.push(share)
            out.append(np.frombuffer(bytes(tree.root()), np.uint8))
        roots.append(np.stack(out))
    return roots[0], roots[1]


def import_extended_data_square(cells, codec=None):
    """rsmt2d.ImportExtendedDataSquare (flattened row-major, None = missing)."""
    n = len(cells)
    w = int(round(n ** 0.5))
    # an all-missing square has no share size to read; use appconsts.ShareSize
    L = max((len(c) for c in cells if c is not None), default=512)
    arr = np.zeros((n, L), np.uint8)
    present = np.zeros(n, np.uint8)
    for i, c in enumerate(cells):
        if c is not None:
            arr[i] = np.frombuffer(bytes(c), np.uint8)
            present[i] = 1
    return ExtendedDataSquare(arr, w, w // 2, codec, present=present)
