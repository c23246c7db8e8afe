"""pkg/wrapper mirror: ErasuredNamespacedMerkleTree + NewConstructor.

Reference: pkg/wrapper/nmt_wrapper.go (celestia-app @ 2025-02-13).  Push keeps
the reference's argument checks and error order (:93-114); Root() hashes the
pushed leaves on the GPU (libcda cda_nmt_axis_root).  ProveRange (:127-130) of one
tree is host code (hashlib: at most 2k leaves); whole squares get their proofs from
the GPU node export (cda.proof / cda.inclusion).
"""
import hashlib

from . import _native as N
from .appconsts import NAMESPACE_SIZE, PARITY_SHARES_NAMESPACE


class PushError(Exception):
    pass


class ErasuredNamespacedMerkleTree:
    def __init__(self, square_size, axis_index, ctx=None):
        if square_size == 0:
            raise ValueError("cannot create a ErasuredNamespacedMerkleTree of squareSize == 0")
        self.square_size = int(square_size)
        self.axis_index = int(axis_index)
        self.share_index = 0
        self._leaves = []
        self._last_ns = None
        self._ctx = ctx

    def _is_quadrant_zero(self):  # nmt_wrapper.go:138-140
        return self.share_index < self.square_size and self.axis_index < self.square_size

    def push(self, data):
        data = bytes(data)
        if self.axis_index + 1 > 2 * self.square_size or self.share_index + 1 > 2 * self.square_size:
            raise PushError(f"pushed past predetermined square size: boundary at {2 * self.square_size} "
                            f"index at {self.axis_index} {self.share_index}")
        if len(data) < NAMESPACE_SIZE:
            raise PushError("data is too short to contain namespace ID")
        ns = data[:NAMESPACE_SIZE] if self._is_quadrant_zero() else PARITY_SHARES_NAMESPACE
        if self._last_ns is not None and ns < self._last_ns:  # nmt ErrInvalidPushOrder
            raise PushError(f"pushed data has smaller namespace than previous: last {self._last_ns.hex()} "
                            f"pushed {ns.hex()}")
        self._last_ns = ns
        self._leaves.append(data)
        self.share_index += 1

    def root(self):
        ctx = self._ctx or N.default_context()
        return ctx.nmt_axis_root(self.square_size, self.axis_index, self._leaves)

    def _leaf_nodes(self):
        out = []
        for i, data in enumerate(self._leaves):
            q0 = i < self.square_size and self.axis_index < self.square_size
            ns = data[:NAMESPACE_SIZE] if q0 else PARITY_SHARES_NAMESPACE
            out.append(ns + ns + hashlib.sha256(b"\x00" + ns + data).digest())
        return out

    def prove_range(self, start, end):
        """ProveRange(start, end) (:127-130 -> nmt Tree.ProveRange): the inclusion proof of leaves [start, end), its
        nodes the roots of the subtrees outside the range, left to right (cda.proof.NMTProof)."""
        from .proof import NMTProof, ProofError, _split_point
        n = len(self._leaves)
        if start < 0 or start >= end or end > n:
            raise ProofError("invalid range")
        leaves = self._leaf_nodes()
        parity = PARITY_SHARES_NAMESPACE
        nodes = []

        def node(left, right):  # nmt HashNode with IgnoreMaxNamespace(true)
            mx = left[NAMESPACE_SIZE:2 * NAMESPACE_SIZE] if right[:NAMESPACE_SIZE] == parity else \
                right[NAMESPACE_SIZE:2 * NAMESPACE_SIZE]
            return left[:NAMESPACE_SIZE] + mx + hashlib.sha256(b"\x01" + left + right).digest()

        def rec(lo, hi, include):
            if lo >= n:
                return None
            if hi - lo == 1:
                if include and not start <= lo < end:
                    nodes.append(leaves[lo])
                return leaves[lo]
            inner = include and not (hi <= start or lo >= end)
            k = _split_point(hi - lo)
            left, right = rec(lo, lo + k, inner), rec(lo + k, hi, inner)
            h = left if right is None else node(left, right)
            if include and not inner:
                nodes.append(h)
            return h

        rec(0, max(1, _split_point(n) * 2), True)
        return NMTProof(start, end, nodes)


def new_erasured_namespaced_merkle_tree(square_size, axis_index, ctx=None):
    return ErasuredNamespacedMerkleTree(square_size, axis_index, ctx)


def new_constructor(square_size, ctx=None):
    """wrapper.NewConstructor(squareSize) rsmt2d.TreeConstructorFn."""

    def new_tree(axis, axis_index):
        return ErasuredNamespacedMerkleTree(square_size, axis_index, ctx)

    # marks the constructor whose trees the fused device path (cda_extend_commit) computes itself
    new_tree.cda_erasured_square_size = int(square_size)
    return new_tree
