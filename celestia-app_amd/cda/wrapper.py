"""pkg/wrapper mirror: ErasuredNamespacedMerkleTree + NewConstructor.

Reference: pkg/wrapper/nmt_wrapper.go (celestia-app @ 2025-02-13).  Push keeps
the reference's argument checks and error order (:93-114); Root() hashes the
pushed leaves on the GPU (libcda cda_nmt_axis_root).
"""
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


def new_erasured_namespaced_merkle_tree(square_size, axis_index, ctx=None):
    return ErasuredNamespacedMerkleTree(square_size, axis_index, ctx)


def new_constructor(square_size, ctx=None):
    """wrapper.NewConstructor(squareSize) rsmt2d.TreeConstructorFn."""

    def new_tree(axis, axis_index):
        return ErasuredNamespacedMerkleTree(square_size, axis_index, ctx)

    # marks the constructor whose trees the fused device path (cda_extend_commit) computes itself
    new_tree.cda_erasured_square_size = int(square_size)
    return new_tree
