"""Blob share commitments and subtree-root paths (celestia-app @ 2025-02-13).

Mirrors go-square v1.0.1's inclusion package (go.mod:9, not vendored; rules in
specs/src/specs/data_square_layout.md:38-58, sparse shares in shares.md:31-81) as
called from x/blob/types/payforblob.go:53 (CreateCommitments) and blob_tx.go:98
(CreateCommitment), and celestia-app's pkg/inclusion (paths.go, nmt_caching.go,
get_commit.go). Path planning is host logic; every hash runs in libcda
(cda_blob_commitments, cda_extend_commit_nodes, cda_merkle_roots).
"""
import math
from dataclasses import dataclass, field

from . import _native as N
from . import appconsts

WALK_LEFT, WALK_RIGHT = False, True  # pkg/inclusion/nmt_caching.go:17-20
FIRST_SPARSE_SHARE_CONTENT_SIZE = appconsts.SHARE_SIZE - appconsts.NAMESPACE_SIZE - 1 - 4  # 478
CONTINUATION_SPARSE_SHARE_CONTENT_SIZE = appconsts.SHARE_SIZE - appconsts.NAMESPACE_SIZE - 1  # 482


class InclusionError(Exception):
    pass


def round_up_power_of_two(x):
    r = 1
    while r < x:
        r <<= 1
    return r


def round_down_power_of_two(x):
    if x <= 0:
        raise InclusionError("input must be positive")
    r = 1
    while r * 2 <= x:
        r <<= 1
    return r


def round_up_by_multiple_of(cursor, v):
    return cursor if cursor % v == 0 else (cursor // v + 1) * v


def sparse_shares_needed(sequence_len):
    """shares.SparseSharesNeeded (shares.md:31-60: 478 data bytes in the first share, 482 after)."""
    if sequence_len == 0:
        return 0
    if sequence_len <= FIRST_SPARSE_SHARE_CONTENT_SIZE:
        return 1
    rest = sequence_len - FIRST_SPARSE_SHARE_CONTENT_SIZE
    return 1 + -(-rest // CONTINUATION_SPARSE_SHARE_CONTENT_SIZE)


def blob_min_square_size(share_count):
    """inclusion.BlobMinSquareSize: smallest power-of-two square the blob fits in."""
    return round_up_power_of_two(math.ceil(math.sqrt(share_count)))


def sub_tree_width(share_count, subtree_root_threshold):
    """inclusion.SubTreeWidth (data_square_layout.md:53, ADR-013)."""
    s = share_count // subtree_root_threshold + (1 if share_count % subtree_root_threshold else 0)
    return min(round_up_power_of_two(s), blob_min_square_size(share_count))


def next_share_index(cursor, blob_share_len, subtree_root_threshold):
    """inclusion.NextShareIndex: the next index a blob of this length may start at."""
    return round_up_by_multiple_of(cursor, sub_tree_width(blob_share_len, subtree_root_threshold))


def merkle_mountain_range_sizes(total_size, max_tree_size):
    """inclusion.MerkleMountainRangeSizes: max-size mountains, then decreasing powers of two."""
    sizes = []
    while total_size:
        t = max_tree_size if total_size >= max_tree_size else round_down_power_of_two(total_size)
        sizes.append(t)
        total_size -= t
    return sizes


@dataclass
class Blob:
    """go-square blob.Blob: namespace = version byte ‖ 28-byte ID."""
    namespace: bytes
    data: bytes
    share_version: int = appconsts.SHARE_VERSION_ZERO


def create_commitments(blobs, subtree_root_threshold=appconsts.SUBTREE_ROOT_THRESHOLD, ctx=None):
    """inclusion.CreateCommitments: one 32-byte share commitment per blob, all blobs in one GPU call."""
    ctx = ctx or N.default_context()
    return ctx.blob_commitments([b.namespace for b in blobs], [b.data for b in blobs],
                                [b.share_version for b in blobs], subtree_root_threshold)


def create_commitment(blob, subtree_root_threshold=appconsts.SUBTREE_ROOT_THRESHOLD, ctx=None):
    """inclusion.CreateCommitment."""
    return create_commitments([blob], subtree_root_threshold, ctx)[0]


# ---- pkg/inclusion/paths.go ----------------------------------------------------------------
@dataclass(frozen=True)
class Coord:
    """A tree node by depth (root = 0) and position (leftmost = 0), paths.go:68-85."""
    depth: int
    position: int

    def climb(self):
        return Coord(self.depth - 1, self.position // 2)

    def can_climb_right(self, min_depth):
        return self.position % 2 == 0 and self.depth > min_depth


@dataclass
class Path:
    instructions: list = field(default_factory=list)
    row: int = 0


def calculate_subtree_root_coordinates(max_depth, min_depth, start, end):
    """calculateSubTreeRootCoordinates (paths.go:108-173)."""
    coords = []
    leaf = start
    node = Coord(max_depth, start)
    last_node, last_leaf, node_range = node, leaf, 1
    while True:
        if leaf + 1 == end:
            coords.append(node)
            return coords
        if leaf + 1 > end:
            coords.append(last_node)
            leaf = last_leaf + 1
        elif not node.can_climb_right(min_depth):
            coords.append(node)
            leaf += 1
        else:
            last_leaf, last_node = leaf, node
            leaf += node_range
            node_range *= 2
            node = node.climb()
            continue
        last_node, last_leaf = node, leaf  # reset()
        node, node_range = Coord(max_depth, leaf), 1


def gen_subtree_root_path(depth, pos):
    """genSubTreeRootPath (paths.go:54-66): bits of pos from the top, 0 = left."""
    return [WALK_RIGHT if pos & (1 << i) else WALK_LEFT for i in range(depth - 1, -1, -1)]


def calculate_commitment_paths(square_size, start, blob_share_len, subtree_root_threshold):
    """calculateCommitmentPaths (paths.go:16-47)."""
    start = next_share_index(start, blob_share_len, subtree_root_threshold)
    start_row, end_row = start // square_size, (start + blob_share_len - 1) // square_size
    norm_start = start % square_size
    norm_end = (start + blob_share_len) - end_row * square_size
    max_depth = int(math.log2(square_size))
    min_depth = max_depth - int(math.log2(sub_tree_width(blob_share_len, subtree_root_threshold)))
    paths = []
    for i in range(start_row, end_row + 1):
        s = norm_start if i == start_row else 0
        e = norm_end if i == end_row else square_size
        for c in calculate_subtree_root_coordinates(max_depth, min_depth, s, e):
            paths.append(Path(gen_subtree_root_path(c.depth, c.position), i))
    return paths


# ---- pkg/inclusion/nmt_caching.go + get_commit.go --------------------------------------------
class EDSSubTreeRootCacher:
    """EDSSubTreeRootCacher (nmt_caching.go:76-124) over the row trees' inner nodes.

    The reference records every inner node through nmt's NodeVisitor while rsmt2d
    builds the row trees, keyed by hash. Here the GPU exports every level of every
    row tree in one call (cda_extend_commit_nodes), and a walk is an index lookup.
    row_nodes: (2k, 4k-1, 90) — per row the leaves first, then each level up to the root.
    """

    def __init__(self, square_size, row_nodes):
        self.square_size = int(square_size)
        self.row_nodes = row_nodes

    @classmethod
    def from_shares(cls, shares, ctx=None):
        """ExtendShares with the cacher as tree constructor + NewDataAvailabilityHeader -> (cacher, dah)."""
        import numpy as np
        from .da import DataAvailabilityHeader
        ctx = ctx or N.default_context()
        arr = np.stack([np.frombuffer(bytes(s), np.uint8) for s in shares])
        out = ctx.extend_commit_nodes(arr, rows=True, cols=False, dah_tree=False)
        k = int(round(len(shares) ** 0.5))
        dah = DataAvailabilityHeader(list(out["row_roots"]), list(out["col_roots"]), ctx=ctx)
        dah._hash = out["dah"]
        return cls(k, out["row_nodes"]), dah

    def get_sub_tree_root(self, dah, row, path):
        """getSubTreeRoot: walk `path` (False = left) down row `row`'s tree from its root."""
        if len(self.row_nodes) != len(dah.row_roots):
            raise InclusionError(f"data availability header has unexpected number of row roots: expected "
                                 f"{len(self.row_nodes)} got {len(dah.row_roots)}")
        if row >= len(self.row_nodes):
            raise InclusionError(f"row exceeds range of cache: max {len(self.row_nodes)} got {row}")
        w = 2 * self.square_size
        levels = w.bit_length() - 1
        if len(path) > levels:
            raise InclusionError("did not find sub tree root")
        pos = 0
        for step in path:
            pos = 2 * pos + (1 if step else 0)
        h = levels - len(path)
        off = sum(w >> i for i in range(h))
        return bytes(self.row_nodes[row][off + pos])


def get_commitment(cacher, dah, start, blob_share_len, subtree_root_threshold, ctx=None):
    """GetCommitment (get_commit.go:12-30): RFC-6962 root of the blob's subtree roots in the ODS half."""
    square_size = len(dah.row_roots) // 2
    if start + blob_share_len > square_size * square_size:
        raise InclusionError("cannot get commitment for blob that doesn't fit in square")
    paths = calculate_commitment_paths(square_size, start, blob_share_len, subtree_root_threshold)
    roots = [cacher.get_sub_tree_root(dah, p.row, [WALK_LEFT] + p.instructions) for p in paths]
    ctx = ctx or N.default_context()
    return ctx.merkle_roots([roots])[0]
