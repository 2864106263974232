"""Mirror of go-square v1.1.0 ``square`` (Construct / Build) over libcda.so.

Reference call sites: app/prepare_proposal.go:50-53 (Build),
app/process_proposal.go:122-126 and app/extend_block.go:16-20 (Construct);
the Builder / Export sequence is the one the reference's malicious copy
spells out (test/util/malicious/out_of_order_builder.go:24-161).  The layout
is planned by the library's host code, the shares are written on the GPU
(no CPU fallback).  Errors carry go-square's messages (``SquareError``).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import NMT_ROOT_SIZE, SHARE_SIZE, default_context, ptr

SQUARE_SIZE_UPPER_BOUND = 128      # pkg/appconsts/v1/app_consts.go:5
SUBTREE_ROOT_THRESHOLD = 64        # pkg/appconsts/v1/app_consts.go:6


class Square(list):
    """square.Square: the k*k shares (512-byte ``bytes``), row-major."""

    def size(self) -> int:
        k = 1
        while k * k < len(self):
            k <<= 1
        return k

    def to_bytes(self) -> bytes:
        """shares.ToBytes, flattened."""
        return b"".join(self)


def _flatten(txs):
    """One flat, writable tx buffer (never empty: a trailing 0 byte) and the
    n + 1 offsets.  One copy of the bytes: np.concatenate of views for blocks
    of few (large) txs, bytes.join for many small ones (per-item cost)."""
    off = np.zeros(len(txs) + 1, dtype=np.uint64)
    np.cumsum(np.fromiter(map(len, txs), dtype=np.uint64, count=len(txs)), out=off[1:])
    if len(txs) <= 512:
        buf = np.concatenate([np.frombuffer(t, dtype=np.uint8) for t in txs] + [np.zeros(1, dtype=np.uint8)])
    else:
        buf = np.frombuffer(bytearray(b"".join(list(txs) + [b"\0"])), dtype=np.uint8)
    return buf, off


def _u64p(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint64))


def layout(txs, max_square_size: int = SQUARE_SIZE_UPPER_BOUND, subtree_root_threshold: int = SUBTREE_ROOT_THRESHOLD,
           build: bool = False):
    """Host-only plan: (square size, kept tx indexes, blob share indexes)."""
    L = _lib.load()
    buf, off = _flatten(txs)
    k = C.c_uint32()
    kept = (C.c_uint32 * max(1, len(txs)))()
    n_kept = C.c_uint32()
    cap = 1 << 16
    idx = (C.c_uint32 * cap)()
    n_idx = C.c_uint32()
    rc = L.cda_square_layout(None, ptr(buf), _u64p(off), len(txs), max_square_size, subtree_root_threshold,
                             _lib.CDA_SQUARE_BUILD if build else _lib.CDA_SQUARE_CONSTRUCT, C.byref(k), kept,
                             C.byref(n_kept), idx, cap, C.byref(n_idx))
    if rc != _lib.CDA_OK:
        msg = L.cda_last_error(None).decode()
        raise (_lib.SquareError if rc == _lib.CDA_ERR_SQUARE else _lib.CdaError)(rc, msg)
    return k.value, list(kept[:n_kept.value]), list(idx[:n_idx.value])


def _construct(txs, max_square_size, threshold, mode, ctx=None):
    ctx = ctx or default_context()
    buf, off = _flatten(txs)
    cap = max_square_size * max_square_size * SHARE_SIZE
    ods = np.empty(cap, dtype=np.uint8)
    k = C.c_uint32()
    kept = (C.c_uint32 * max(1, len(txs)))()
    n_kept = C.c_uint32()
    ctx.check(ctx.lib.cda_square_construct(ctx.h, ptr(buf), _u64p(off), len(txs), max_square_size, threshold, mode,
                                           ptr(ods), cap, C.byref(k), kept, C.byref(n_kept)))
    n = k.value * k.value
    raw = ods[:n * SHARE_SIZE].tobytes()
    sq = Square(raw[i * SHARE_SIZE:(i + 1) * SHARE_SIZE] for i in range(n))
    return sq, list(kept[:n_kept.value])


def construct(txs, max_square_size: int = SQUARE_SIZE_UPPER_BOUND,
              subtree_root_threshold: int = SUBTREE_ROOT_THRESHOLD, ctx=None) -> Square:
    """square.Construct: the exact, ordered txs of a block -> Square."""
    return _construct(txs, max_square_size, subtree_root_threshold, _lib.CDA_SQUARE_CONSTRUCT, ctx)[0]


def build(txs, max_square_size: int = SQUARE_SIZE_UPPER_BOUND, subtree_root_threshold: int = SUBTREE_ROOT_THRESHOLD,
          ctx=None):
    """square.Build: prioritised txs -> (Square, the txs in it: normal then blob txs)."""
    sq, kept = _construct(txs, max_square_size, subtree_root_threshold, _lib.CDA_SQUARE_BUILD, ctx)
    return sq, [txs[i] for i in kept]


def construct_extend_dah(txs, max_square_size: int = SQUARE_SIZE_UPPER_BOUND,
                         subtree_root_threshold: int = SUBTREE_ROOT_THRESHOLD, build_mode: bool = False,
                         want_eds: bool = False, ctx=None):
    """Construct (or Build) + ExtendShares + NewDataAvailabilityHeader in one
    device submission.  Returns (k, eds bytes or None, row_roots, col_roots,
    data_root, kept tx indexes)."""
    ctx = ctx or default_context()
    buf, off = _flatten(txs)
    w_max = 2 * max_square_size
    eds = np.empty(w_max * w_max * SHARE_SIZE, dtype=np.uint8) if want_eds else None
    rows = np.empty(w_max * NMT_ROOT_SIZE, dtype=np.uint8)
    cols = np.empty(w_max * NMT_ROOT_SIZE, dtype=np.uint8)
    root = np.empty(32, dtype=np.uint8)
    k = C.c_uint32()
    kept = (C.c_uint32 * max(1, len(txs)))()
    n_kept = C.c_uint32()
    mode = _lib.CDA_SQUARE_BUILD if build_mode else _lib.CDA_SQUARE_CONSTRUCT
    ctx.check(ctx.lib.cda_construct_extend_dah(ctx.h, ptr(buf), _u64p(off), len(txs), max_square_size,
                                               subtree_root_threshold, mode, ptr(eds),
                                               0 if eds is None else eds.size, ptr(rows), ptr(cols), rows.size,
                                               ptr(root), C.byref(k), kept, C.byref(n_kept)))
    w = 2 * k.value
    rr = [rows[i * NMT_ROOT_SIZE:(i + 1) * NMT_ROOT_SIZE].tobytes() for i in range(w)]
    cr = [cols[i * NMT_ROOT_SIZE:(i + 1) * NMT_ROOT_SIZE].tobytes() for i in range(w)]
    e = eds[:w * w * SHARE_SIZE].tobytes() if eds is not None else None
    return k.value, e, rr, cr, root.tobytes(), list(kept[:n_kept.value])
