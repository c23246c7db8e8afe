"""rsmt2d-shaped API (github.com/celestiaorg/rsmt2d v0.12.0, go.mod:13) over libcda.

Mirrors the pieces celestia-app uses: the Codec interface (LeoRSCodec,
selected at pkg/appconsts/global_consts.go:92), ComputeExtendedDataSquare,
ExtendedDataSquare.{RowRoots,ColRoots,Row,Col,GetCell,SetCell,Flattened,Width},
Repair and its error types.  All arithmetic runs in libcda on the GPU.
"""
from concurrent.futures import ThreadPoolExecutor

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
        if not any(s is not None for s in shards):  # go/cda Codec.Decode: no shard to read a size from
            raise N.CdaError(N.E_TOO_FEW)
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




def compute_extended_data_square_axes(data, codec=None, tree_constructor=None, workers=8):
    """rsmt2d.ComputeExtendedDataSquare as upstream rsmt2d v0.12.0 runs it on an unpatched caller -- the shape every
    rsmt2d user gets with appconsts.DefaultCodec = the GPU codec (go/pkg_da/extend_rocm.go): erasureExtendSquare
    encodes one axis per task through codec.encode (row i then column i for i < k, then rows k..2k-1: Q3 = Enc(Q2
    rows)), and computeRoots pushes each axis into a tree from `tree_constructor` (default wrapper.NewConstructor(k),
    whose Root is cda_nmt_axis_root) and takes its Root, one task per index.  `workers` threads stand in for the
    goroutines; concurrent calls meet in libcda's axis queue (axisq.cpp).  Same bytes as compute_extended_data_square,
    which runs the whole square as one fused call."""
    from . import wrapper
    codec = codec or LeoRSCodec()
    if len(data) > codec.max_chunks():
        raise ValueError("number of chunks exceeds the maximum")
    k = int(round(len(data) ** 0.5))
    if k * k != len(data):
        raise ValueError("number of chunks must be a square number")
    w = 2 * k
    L = len(bytes(data[0])) if k else 512
    cells = np.zeros((w * w, L), np.uint8)
    grid = cells.reshape(w, w, L)
    for i, d in enumerate(data):
        grid[i // k, i % k] = np.frombuffer(bytes(d), np.uint8)
    tree_constructor = tree_constructor or wrapper.new_constructor(k, codec.ctx)

    def extend_row(i):  # erasureExtendRow: Encode(rowSlice(i, 0, k)) -> setRowSlice(i, k, parity)
        par = codec.encode([grid[i, j].tobytes() for j in range(k)])
        for j, p in enumerate(par):
            grid[i, k + j] = np.frombuffer(p, np.uint8)

    def extend_col(i):  # erasureExtendCol: Encode(colSlice(0, i, k)) -> setColSlice(k, i, parity)
        par = codec.encode([grid[j, i].tobytes() for j in range(k)])
        for j, p in enumerate(par):
            grid[k + j, i] = np.frombuffer(p, np.uint8)

    with ThreadPoolExecutor(max_workers=workers) as ex:
        list(ex.map(lambda i: (extend_row(i), extend_col(i)), range(k)))
        list(ex.map(lambda i: extend_row(k + i), range(k)))
        sq = ExtendedDataSquare(cells, w, k, codec)
        roots = list(ex.map(lambda i: (_axis_root(sq, tree_constructor, ROW, i),
                                       _axis_root(sq, tree_constructor, COL, i)), range(w)))
    sq._row_roots = np.stack([np.frombuffer(r, np.uint8) for r, _ in roots])
    sq._col_roots = np.stack([np.frombuffer(c, np.uint8) for _, c in roots])
    return sq


def _axis_root(sq, tree_constructor, axis, i, cells=None):
    """rsmt2d computeSharesRoot: a fresh tree from the constructor, the axis's cells pushed in order, Root()."""
    tree = tree_constructor(axis, i)
    for share in (cells if cells is not None else (sq.row(i) if axis == ROW else sq.col(i))):
        tree.push(share)
    return bytes(tree.root())


def repair_axes(sq, row_roots, col_roots, tree_constructor=None, workers=8):
    """(*ExtendedDataSquare).Repair as upstream rsmt2d v0.12.0 runs it over the codec and tree seams -- what
    celestia-node's Repair of a square returned by cda.ExtendShares reaches: prerepairSanityCheck (every complete
    axis's root against the given roots and its parity against codec.encode of its data half, one task per axis),
    then solveCrossword sequentially: for each index, row then column, an incomplete axis is rebuilt with codec.decode
    when it can be, its root checked, the roots of the orthogonal axes it completes checked, and its cells set; sweeps
    repeat until the square is complete (ok) or a sweep makes no progress (ErrUnrepairableDataSquare).  A mismatch
    raises ErrByzantineData(axis, index) with the square left as repaired so far.  Same result as sq.repair (one
    cda_repair call), one device round trip per axis instead."""
    from . import wrapper
    w, k = sq.width(), sq.original_data_width
    tree_constructor = tree_constructor or wrapper.new_constructor(k, sq.codec.ctx)
    rr = [bytes(r) for r in row_roots]
    cr = [bytes(c) for c in col_roots]
    want = {ROW: rr, COL: cr}

    def vec(axis, i):
        return sq.row(i) if axis == ROW else sq.col(i)

    def complete(axis, i, skip=-1):
        return all(s is not None for j, s in enumerate(vec(axis, i)) if j != skip)

    def root_ok(axis, i, cells):
        try:
            return _axis_root(sq, tree_constructor, axis, i, cells) == want[axis][i]
        except Exception:  # a tree that cannot be built (push order) does not match its root
            return False

    def sanity(i):
        rowc, colc = complete(ROW, i), complete(COL, i)
        for step, axis in enumerate((ROW, COL, ROW, COL)):
            if not (rowc if axis == ROW else colc):
                continue
            v = vec(axis, i)
            ok = root_ok(axis, i, v) if step < 2 else \
                b"".join(sq.codec.encode(v[:k])) == b"".join(v[k:])
            if not ok:
                return i * 4 + step
        return None

    with ThreadPoolExecutor(max_workers=workers) as ex:
        bad = [b for b in ex.map(sanity, range(w)) if b is not None]
    if bad:
        b = min(bad)
        raise ErrByzantineData(ROW if b % 2 == 0 else COL, b // 4)

    def solve(axis, i):  # -> (solved, progress)
        if complete(axis, i):
            return True, False
        shares = vec(axis, i)
        try:
            rebuilt = sq.codec.decode(shares)
        except N.CdaError as e:
            if e.code == N.E_TOO_FEW:
                return False, False
            raise
        if not root_ok(axis, i, rebuilt):
            raise ErrByzantineData(axis, i, shares)
        other = COL if axis == ROW else ROW
        for j in range(w):
            cell = (i, j) if axis == ROW else (j, i)
            if sq.get_cell(*cell) is not None or not complete(other, j, skip=i):
                continue
            ov = vec(other, j)
            ov[i] = rebuilt[j]
            if not root_ok(other, j, ov):
                raise ErrByzantineData(other, j, vec(other, j))
        for j in range(w):
            cell = (i, j) if axis == ROW else (j, i)
            if sq.get_cell(*cell) is None:
                sq.set_cell(*cell, rebuilt[j])
        return True, True

    while True:
        solved, progress = True, False
        for i in range(w):
            for axis in (ROW, COL):
                s, p = solve(axis, i)
                solved, progress = solved and s, progress or p
        if solved:
            break
        if not progress:
            raise ErrUnrepairableDataSquare()
    sq._row_roots = np.stack([np.frombuffer(r, np.uint8) for r in rr])
    sq._col_roots = np.stack([np.frombuffer(c, np.uint8) for c in cr])


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
