"""Mirror of the rsmt2d v0.14.0 surface used by celestia-app's DA path.

rsmt2d is an EXT Go module (pinned at /root/reference/go.mod:13); celestia-app
reaches it through pkg/da/data_availability_header.go:45,49,74 and
pkg/appconsts/global_consts.go:92 (DefaultCodec = rsmt2d.NewLeoRSCodec).
Names and error texts follow the Go API; every computation runs on the GPU
through libcda.so.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import SHARE_SIZE, ByzantineDataError, CdaError, PushOrderError, UnrepairableError, default_context, ptr

ROW = 0
COL = 1
LEOPARD = "Leopard"


ErrByzantineData = ByzantineDataError
ErrUnrepairableDataSquare = UnrepairableError


class ErrUnevenChunks(ValueError):
    def __init__(self):
        super().__init__("non-nil chunks not all of equal size")


def _as_shares(data) -> np.ndarray:
    if isinstance(data, np.ndarray):
        a = np.ascontiguousarray(data, dtype=np.uint8)
        return a.reshape(a.shape[0], -1) if a.ndim != 2 else a
    data = list(data)
    if not data:
        return np.zeros((0, 0), dtype=np.uint8)
    size = None
    for d in data:
        if d is not None:
            size = len(d)
            break
    for d in data:
        if d is not None and len(d) != size:
            raise ErrUnevenChunks()
    return np.frombuffer(b"".join(bytes(d) for d in data), dtype=np.uint8).reshape(len(data), size).copy()


class LeoRSCodec:
    """rsmt2d.LeoRSCodec (Leopard RS via klauspost/reedsolomon v1.12.1)."""

    def __init__(self, ctx=None):
        self._ctx = ctx

    @property
    def ctx(self):
        return self._ctx or default_context()

    def encode(self, data) -> np.ndarray:
        """Codec.Encode: k data shards -> k parity shards (k a power of two)."""
        shards = _as_shares(data)
        k, L = shards.shape
        parity = np.empty_like(shards)
        self.ctx.check(self.ctx.lib.cda_rs_encode(self.ctx.h, ptr(shards), k, L, 1, ptr(parity)))
        return parity

    def encode_batch(self, codewords: np.ndarray) -> np.ndarray:
        """Encode n independent codewords (n, k, L) in one submission."""
        cw = np.ascontiguousarray(codewords, dtype=np.uint8)
        n, k, L = cw.shape
        parity = np.empty_like(cw)
        self.ctx.check(self.ctx.lib.cda_rs_encode(self.ctx.h, ptr(cw), k, L, n, ptr(parity)))
        return parity

    def decode(self, data):
        """Codec.Decode (reedsolomon Reconstruct): 2k shards, missing ones as
        None; returns all 2k shards (ErrTooFewShards -> UnrepairableError)."""
        data = list(data)
        n = len(data)
        present = np.array([d is not None for d in data], dtype=np.uint8)
        size = next((len(d) for d in data if d is not None), 0)
        filled = _as_shares([d if d is not None else bytes(size) for d in data])
        self.decode_batch(filled[None], present[None])
        return [filled[i].tobytes() for i in range(n)]

    def decode_batch(self, shards: np.ndarray, present: np.ndarray) -> np.ndarray:
        """Reconstruct, in place, n codewords (n, 2k, L) with presence (n, 2k)."""
        n, w, L = shards.shape
        if not shards.flags.c_contiguous or shards.dtype != np.uint8:
            raise ValueError("shards must be a C-contiguous uint8 array")
        pres = np.ascontiguousarray(present, dtype=np.uint8)
        self.ctx.check(self.ctx.lib.cda_rs_decode(self.ctx.h, ptr(shards), ptr(pres), w // 2, L, n))
        return shards

    def max_chunks(self) -> int:
        return 32768 * 32768

    def name(self) -> str:
        return LEOPARD

    def validate_chunk_size(self, chunk_size: int):
        if chunk_size % 64 != 0:
            raise ValueError(f"chunkSize {chunk_size} must be a multiple of 64 bytes")


def new_leo_rs_codec() -> LeoRSCodec:
    return LeoRSCodec()


class ExtendedDataSquare:
    """rsmt2d.ExtendedDataSquare backed by one contiguous (W, W, 512) array.

    Roots are produced by the same GPU submission that extended the square
    (or, for an imported square, by one GPU call on first use) and handed to
    the trees of the constructor, mirroring how the cgo drop-in seeds
    wrapper.NewConstructor.
    """

    def __init__(self, eds: np.ndarray, codec, tree_fn, roots=None, err: Exception | None = None):
        self._eds = eds
        self.codec = codec
        self.tree_fn = tree_fn
        self._roots = roots
        self._err = err
        # rsmt2d hashes the cells when RowRoots / ColRoots is first called; the
        # roots here come from the extension's own GPU submission, so they
        # hold only while the cells are still the bytes that submission
        # hashed.  The fingerprint of those bytes is checked on first use.
        self._fp = _fingerprint(eds) if (roots is not None or err is not None) else None

    # -- geometry ---------------------------------------------------------
    def width(self) -> int:
        return self._eds.shape[0]

    def original_data_width(self) -> int:
        return self._eds.shape[0] // 2

    def get_cell(self, r: int, c: int) -> bytes:
        return self._eds[r, c].tobytes()

    def row(self, r: int):
        return [self._eds[r, c].tobytes() for c in range(self.width())]

    def col(self, c: int):
        return [self._eds[r, c].tobytes() for r in range(self.width())]

    def flattened(self):
        return [self._eds[r, c].tobytes() for r in range(self.width()) for c in range(self.width())]

    def flattened_ods(self):
        k = self.original_data_width()
        return [self._eds[r, c].tobytes() for r in range(k) for c in range(k)]

    def array(self) -> np.ndarray:
        """Zero-copy view of the EDS as (W, W, 512) uint8."""
        return self._eds

    # -- roots --------------------------------------------------------------
    def _compute_roots(self):
        if self._fp is not None:
            # first use: cells rewritten in place since the extension (same
            # backing array) invalidate the submission's roots, exactly as
            # rsmt2d's computeRoots would hash the new bytes
            if _fingerprint(self._eds) != self._fp:
                self._roots, self._err = None, None
            self._fp = None
        if self._roots is None and self._err is None:
            ctx = getattr(self.codec, "ctx", None) or default_context()
            W = self.width()
            rows = np.empty((W, _lib.NMT_ROOT_SIZE), dtype=np.uint8)
            cols = np.empty((W, _lib.NMT_ROOT_SIZE), dtype=np.uint8)
            root = np.empty(32, dtype=np.uint8)
            flat = np.ascontiguousarray(self._eds)
            try:
                ctx.check(ctx.lib.cda_dah_from_eds(ctx.h, ptr(flat), W, ptr(rows), ptr(cols), ptr(root)))
                self._roots = (rows, cols, root.tobytes())
            except PushOrderError as e:
                self._err = e
        if self._err is not None:
            raise self._err
        return self._roots

    def row_roots(self):
        rows, _, _ = self._compute_roots()
        return self._seed(ROW, rows)

    def col_roots(self):
        _, cols, _ = self._compute_roots()
        return self._seed(COL, cols)

    def _seed(self, axis: int, roots: np.ndarray):
        out = []
        for i in range(roots.shape[0]):
            tree = self.tree_fn(axis, i)
            seed = getattr(tree, "_seed_root", None)
            if seed is not None:
                seed(roots[i].tobytes(), self._eds[i, :] if axis == ROW else self._eds[:, i])
                out.append(tree.root())
            else:   # a foreign Tree implementation: push every cell (rsmt2d getRowRoot)
                cells = self._eds[i, :] if axis == ROW else self._eds[:, i]
                for cell in cells:
                    tree.push(cell.tobytes())
                out.append(tree.root())
        return out

    def data_root(self) -> bytes:
        return self._compute_roots()[2]

    # -- repair -------------------------------------------------------------
    def repair(self, row_roots, col_roots, present=None):
        """ExtendedDataSquare.Repair(rowRoots, colRoots).

        ``present`` (W, W) marks the cells that are held (rsmt2d: non-nil
        cells); by default every cell is.  Raises ByzantineDataError (with
        .axis / .index), UnrepairableError or CdaError("bad root input ...").
        The square is updated in place, also on an error.
        """
        W = self.width()
        if len(row_roots) != W or len(col_roots) != W:
            raise ValueError("number of roots does not match the square width")
        if present is None:
            present = np.ones((W, W), dtype=np.uint8)
        pres = np.ascontiguousarray(present, dtype=np.uint8)
        rows = np.frombuffer(b"".join(bytes(r) for r in row_roots), dtype=np.uint8)
        cols = np.frombuffer(b"".join(bytes(c) for c in col_roots), dtype=np.uint8)
        ctx = getattr(self.codec, "ctx", None) or default_context()
        if not self._eds.flags.c_contiguous:
            self._eds = np.ascontiguousarray(self._eds)
        axis = C.c_int32(-1)
        index = C.c_uint32(0)
        rc = ctx.lib.cda_repair(ctx.h, ptr(self._eds), ptr(pres), W, ptr(rows), ptr(cols), C.byref(axis),
                                C.byref(index))
        self._roots, self._err, self._fp = None, None, None
        if rc == _lib.CDA_ERR_BYZANTINE:
            raise ByzantineDataError(rc, ctx.lib.cda_last_error(ctx.h).decode(), axis.value, index.value)
        ctx.check(rc)


def _fingerprint(a: np.ndarray) -> bytes:
    """128-bit content fingerprint of a square's cells (xxh3, ~5 GB/s on one
    core; blake2b when the xxhash module is absent)."""
    buf = np.ascontiguousarray(a)
    try:
        import xxhash
        return xxhash.xxh3_128_digest(buf)
    except ImportError:
        import hashlib
        return hashlib.blake2b(buf, digest_size=16).digest()


def new_extended_data_square_with_missing(eds: np.ndarray, present: np.ndarray, codec, tree_fn):
    """A square as a sampling node holds it: cells with present == 0 are
    zeroed (rsmt2d nil cells)."""
    eds = np.array(eds, dtype=np.uint8, copy=True)
    eds[np.asarray(present) == 0] = 0
    return ExtendedDataSquare(eds, codec, tree_fn)


def _square_k(n: int) -> int:
    k = int(round(n ** 0.5))
    if k * k != n:
        raise ValueError("number of chunks must be a square number")
    return k


def compute_extended_data_square(data, codec: LeoRSCodec, tree_fn) -> ExtendedDataSquare:
    """rsmt2d.ComputeExtendedDataSquare: extend and (in the same GPU
    submission) compute all 4k NMT roots and the data root."""
    shares = _as_shares(data)
    if shares.shape[0] > codec.max_chunks():
        raise ValueError("number of chunks exceeds the maximum")
    codec.validate_chunk_size(shares.shape[1])
    n = shares.shape[0]
    k = _square_k(n)
    if shares.shape[1] != SHARE_SIZE:
        raise CdaError(_lib.CDA_ERR_UNSUPPORTED, f"chunk size {shares.shape[1]} unsupported (shares are "
                                                 f"{SHARE_SIZE} bytes)")
    ctx = codec.ctx
    W = 2 * k
    eds = np.empty((W, W, SHARE_SIZE), dtype=np.uint8)
    rows = np.empty((W, _lib.NMT_ROOT_SIZE), dtype=np.uint8)
    cols = np.empty((W, _lib.NMT_ROOT_SIZE), dtype=np.uint8)
    root = np.empty(32, dtype=np.uint8)
    rc = ctx.lib.cda_extend_dah(ctx.h, ptr(shares), n, ptr(eds), ptr(rows), ptr(cols), ptr(root))
    if rc == _lib.CDA_ERR_PUSH_ORDER:
        try:
            ctx.check(rc)
        except PushOrderError as e:
            return ExtendedDataSquare(eds, codec, tree_fn, err=e)
    ctx.check(rc)
    return ExtendedDataSquare(eds, codec, tree_fn, roots=(rows, cols, root.tobytes()))


def import_extended_data_square(data, codec: LeoRSCodec, tree_fn) -> ExtendedDataSquare:
    """rsmt2d.ImportExtendedDataSquare: wrap an already-extended square."""
    shares = _as_shares(data)
    codec.validate_chunk_size(shares.shape[1])
    W = _square_k(shares.shape[0])
    return ExtendedDataSquare(shares.reshape(W, W, shares.shape[1]), codec, tree_fn)
