"""Mirror of pkg/wrapper (ErasuredNamespacedMerkleTree, NewConstructor).

Reference: /root/reference/pkg/wrapper/nmt_wrapper.go.  Push validates exactly
like the reference (:93-114 and nmt's push order) and keeps the pushed cells;
Root (:118-124) and ProveRange (:126-129) hash them on the GPU
(cda_nmt_axis_root / cda_nmt_prove_range).  A tree handed out by an
ExtendedDataSquare is pre-seeded with the root the square's own GPU submission
computed (the cgo drop-in does the same): the seed is used
only while the tree holds exactly the bytes it was seeded for -- a push of any
other bytes drops it and the root is recomputed from what was pushed.  Bytes,
not buffers: seed() keeps a private copy of the seeded cells, so a cell
rewritten in place after seeding (same backing array) is seen as different;
the square's own trees are seeded only after ExtendedDataSquare has checked
its cells against the extension's fingerprint (rsmt2d.py).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import NAMESPACE_SIZE, NMT_ROOT_SIZE, default_context, ptr

PARITY_SHARES_NAMESPACE = b"\xff" * NAMESPACE_SIZE   # go-square namespace.ParitySharesNamespace
EMPTY_ROOT = b"\x00" * (2 * NAMESPACE_SIZE) + bytes.fromhex(
    "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855")  # NmtHasher.EmptyRoot


class ErasuredNamespacedMerkleTree:
    def __init__(self, square_size: int, axis_index: int, ctx=None):
        if square_size == 0:
            raise ValueError("cannot create a ErasuredNamespacedMerkleTree of squareSize == 0")
        self.square_size = square_size
        self.axis_index = axis_index
        self.share_index = 0
        self._ctx = ctx
        self._last_ns = None
        self._cells = []            # pushed data, in order (nmt keeps every leaf)
        self._seed = None           # (root, cells) from the square's GPU submission
        self._root = None

    @property
    def ctx(self):
        return self._ctx or default_context()

    def _is_quadrant_zero(self) -> bool:
        return self.share_index < self.square_size and self.axis_index < self.square_size

    def push(self, data):
        """Push (:93-114): bounds, namespace length, nmt push order."""
        if self.axis_index + 1 > 2 * self.square_size or self.share_index + 1 > 2 * self.square_size:
            raise ValueError(f"pushed past predetermined square size: boundary at {2 * self.square_size} "
                             f"index at {self.axis_index} {self.share_index}")
        if len(data) < NAMESPACE_SIZE:
            raise ValueError("data is too short to contain namespace ID")
        ns = bytes(data[:NAMESPACE_SIZE]) if self._is_quadrant_zero() else PARITY_SHARES_NAMESPACE
        if self._last_ns is not None and ns < self._last_ns:
            raise ValueError("pushed data has to be lexicographically ordered by namespace IDs: "
                             f"last namespace: {self._last_ns.hex()}, pushed: {ns.hex()}")
        if self._seed is not None:
            cells = self._seed[1]
            i = self.share_index
            if not (i < len(cells) and bytes(data) == bytes(cells[i])):
                self._seed = None   # not the seeded bytes: the GPU root is recomputed
        self._last_ns = ns
        if not isinstance(self._cells, list):
            self._cells = list(self._cells)
        self._cells.append(data)
        self.share_index += 1
        self._root = None

    # -- seeding (rsmt2d.ExtendedDataSquare) ---------------------------------
    def seed(self, root: bytes, cells):
        """Offer the root the square's GPU submission computed for `cells`;
        it is used only if exactly these bytes are pushed (a private copy is
        kept, so rewriting the caller's buffers afterwards drops the seed)."""
        self._seed = (root, [bytes(c) for c in cells])

    def _seed_root(self, root: bytes, cells):
        """Seed and adopt: the tree holds `cells` (the square's own row or
        column, whose bytes the square has just checked against its
        extension's fingerprint) and is rooted at once."""
        self._seed = (root, cells)
        self._cells = cells
        self.share_index = len(cells)
        self._last_ns = PARITY_SHARES_NAMESPACE if len(cells) > self.square_size else None
        self._root = None

    def _flat_cells(self) -> np.ndarray:
        if isinstance(self._cells, np.ndarray):
            return np.ascontiguousarray(self._cells, dtype=np.uint8).reshape(-1)
        lens = {len(c) for c in self._cells}
        if len(lens) != 1:
            raise ValueError("cells of one tree must have equal length")
        return np.ascontiguousarray(np.frombuffer(b"".join(bytes(c) for c in self._cells), dtype=np.uint8))

    def root(self) -> bytes:
        """Root (:118-124)."""
        if self._root is not None:
            return self._root
        if self.share_index == 0:
            return EMPTY_ROOT
        if self._seed is not None and self.share_index == len(self._seed[1]):
            self._root = self._seed[0]
            return self._root
        flat = self._flat_cells()
        out = np.empty(NMT_ROOT_SIZE, dtype=np.uint8)
        ctx = self.ctx
        ctx.check(ctx.lib.cda_nmt_axis_root(ctx.h, ptr(flat), len(self._cells[0]), self.share_index,
                                            self.square_size, self.axis_index, ptr(out)))
        self._root = out.tobytes()
        return self._root

    def prove_range(self, start: int, end: int):
        """ProveRange (:126-129 -> nmt ProveRange): the proof nodes (90 B
        each) of leaves [start, end), maximal subtrees outside the range,
        depth first, left to right."""
        if start < 0 or start >= end or end > self.share_index:
            raise ValueError("invalid proof range")
        flat = self._flat_cells()
        n = self.share_index
        nodes = np.empty(2 * max(1, n.bit_length()) * NMT_ROOT_SIZE, dtype=np.uint8)
        count = C.c_uint32()
        root = np.empty(NMT_ROOT_SIZE, dtype=np.uint8)
        ctx = self.ctx
        ctx.check(ctx.lib.cda_nmt_prove_range(ctx.h, ptr(flat), len(self._cells[0]), n, self.square_size,
                                              self.axis_index, start, end, ptr(nodes), C.byref(count), ptr(root)))
        if self._root is None:
            self._root = root.tobytes()
        return [nodes[i * NMT_ROOT_SIZE:(i + 1) * NMT_ROOT_SIZE].tobytes() for i in range(count.value)]


def new_erasured_namespaced_merkle_tree(square_size: int, axis_index: int, ctx=None) -> ErasuredNamespacedMerkleTree:
    return ErasuredNamespacedMerkleTree(square_size, axis_index, ctx)


def new_constructor(square_size: int, ctx=None):
    """wrapper.NewConstructor: returns a TreeConstructorFn (axis, index) -> Tree."""
    def new_tree(_axis: int, axis_index: int):
        return ErasuredNamespacedMerkleTree(square_size, axis_index, ctx)
    return new_tree


def axis_roots(cells: np.ndarray, square_size: int, axis_indexes, ctx=None) -> np.ndarray:
    """Roots of many standalone trees in one GPU submission
    (cda_nmt_axis_roots): cells (n_trees, n_cells, cell_len) -> (n_trees, 90),
    e.g. every row of a square rebuilt outside ComputeExtendedDataSquare
    (pkg/inclusion/nmt_caching.go:96-109)."""
    ctx = ctx or default_context()
    cells = np.ascontiguousarray(cells, dtype=np.uint8)
    n_trees, n_cells, cell_len = cells.shape
    axes = np.ascontiguousarray(axis_indexes, dtype=np.uint32)
    roots = np.empty((n_trees, NMT_ROOT_SIZE), dtype=np.uint8)
    status = np.empty(n_trees, dtype=np.int32)
    ctx.check(ctx.lib.cda_nmt_axis_roots(ctx.h, ptr(cells), cell_len, n_cells, n_trees, square_size,
                                         axes.ctypes.data_as(C.POINTER(C.c_uint32)), ptr(roots),
                                         status.ctypes.data_as(C.POINTER(C.c_int32))))
    return roots
