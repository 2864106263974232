"""Mirror of pkg/wrapper (ErasuredNamespacedMerkleTree, NewConstructor).

Reference: /root/reference/pkg/wrapper/nmt_wrapper.go.  The constructor's trees
validate every Push exactly like the reference (:93-114, nmt push order) and
return the root computed on the GPU for the whole square by the same
submission that extended it (rsmt2d.ExtendedDataSquare._seed).
"""
from __future__ import annotations

from ._lib import NAMESPACE_SIZE

PARITY_SHARES_NAMESPACE = b"\xff" * NAMESPACE_SIZE   # go-square namespace.ParitySharesNamespace
EMPTY_ROOT = b"\x00" * (2 * NAMESPACE_SIZE) + bytes.fromhex(
    "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855")  # NmtHasher.EmptyRoot


class ErasuredNamespacedMerkleTree:
    def __init__(self, square_size: int, axis_index: int):
        if square_size == 0:
            raise ValueError("cannot create a ErasuredNamespacedMerkleTree of squareSize == 0")
        self.square_size = square_size
        self.axis_index = axis_index
        self.share_index = 0
        self._last_ns = None
        self._root = None

    def _is_quadrant_zero(self) -> bool:
        return self.share_index < self.square_size and self.axis_index < self.square_size

    def push(self, data: bytes):
        if self.axis_index + 1 > 2 * self.square_size or self.share_index + 1 > 2 * self.square_size:
            raise ValueError(f"pushed past predetermined square size: boundary at {2 * self.square_size} "
                             f"index at {self.axis_index} {self.share_index}")
        if len(data) < NAMESPACE_SIZE:
            raise ValueError("data is too short to contain namespace ID")
        ns = bytes(data[:NAMESPACE_SIZE]) if self._is_quadrant_zero() else PARITY_SHARES_NAMESPACE
        if self._last_ns is not None and ns < self._last_ns:
            raise ValueError("pushed data has to be lexicographically ordered by namespace IDs: "
                             f"last namespace: {self._last_ns.hex()}, pushed: {ns.hex()}")
        self._last_ns = ns
        self.share_index += 1
        self._root = None

    def _seed_root(self, root: bytes, cells):
        """Adopt the GPU root for this axis; the cells are pushed for the
        bookkeeping the reference does (indices, namespaces)."""
        self.share_index = len(cells)
        self._last_ns = PARITY_SHARES_NAMESPACE if len(cells) > self.square_size else None
        self._root = root

    def root(self) -> bytes:
        if self._root is not None:
            return self._root
        if self.share_index == 0:
            return EMPTY_ROOT
        raise NotImplementedError("standalone NMT trees are computed per square; use "
                                  "rsmt2d.compute_extended_data_square")


def new_erasured_namespaced_merkle_tree(square_size: int, axis_index: int) -> ErasuredNamespacedMerkleTree:
    return ErasuredNamespacedMerkleTree(square_size, axis_index)


def new_constructor(square_size: int):
    """wrapper.NewConstructor: returns a TreeConstructorFn (axis, index) -> Tree."""
    def new_tree(_axis: int, axis_index: int):
        return ErasuredNamespacedMerkleTree(square_size, axis_index)
    return new_tree
