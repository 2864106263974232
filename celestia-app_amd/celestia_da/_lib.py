"""ctypes binding of libcda.so (include/cda.h).

The HIP library is the only compute path: if it cannot be loaded this module
raises, there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import importlib.util
import os
import sys
import threading

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("CDA_LIB", os.path.join(PKG_ROOT, "libcda.so"))
# The test build (make -C celestia-app_amd test-lib; -DCDA_TESTING): the same
# kernels, plus the test knobs -- fault injection and A/B schedule switches --
# that libcda.so never reads (csrc/knobs.h).  Only tests load it.
TEST_LIB_PATH = os.path.join(PKG_ROOT, "libcda_test.so")

SHARE_SIZE = 512
NAMESPACE_SIZE = 29
NMT_ROOT_SIZE = 90
HASH_SIZE = 32

CDA_OK = 0
CDA_ERR_NOT_POW2 = -1
CDA_ERR_CHUNK_SIZE = -2
CDA_ERR_PUSH_ORDER = -3
CDA_ERR_DEVICE = -4
CDA_ERR_OOM = -5
CDA_ERR_INVALID = -6
CDA_ERR_UNSUPPORTED = -7
CDA_ERR_SQUARE = -8
CDA_ERR_BYZANTINE = -9
CDA_ERR_UNREPAIRABLE = -10
CDA_ERR_COMM = -11

CDA_SQUARE_CONSTRUCT = 0
CDA_SQUARE_BUILD = 1

# cda_extend_dah_batch_ex eds modes (include/cda.h)
CDA_EDS_FULL = 0
CDA_EDS_SKIP_Q0 = 1
CDA_EDS_PARITY = 2

# cda_split_offsets selectors (include/cda.h)
CDA_SPLIT_SEND = 0
CDA_SPLIT_SEND_PIECE = 1
CDA_SPLIT_RECV_PIECE = 2
CDA_SPLIT_BLOCK = 3
CDA_SPLIT_GATHER_SUB = 4
CDA_SPLIT_GATHER_COL = 5
CDA_SPLIT_COMBINE = 6

EXPORTED = (
    "cda_ctx_create", "cda_ctx_destroy", "cda_last_error", "cda_version", "cda_extend_shares",
    "cda_dah_from_eds", "cda_extend_dah", "cda_extend_dah_batch", "cda_extend_dah_device",
    "cda_extend_dah_inplace_device", "cda_reserve",
    "cda_rs_encode", "cda_data_root", "cda_push_order_detail", "cda_push_order_detail_at", "cda_set_profiling", "cda_stage_times",
    "cda_split_rows", "cda_split_cols", "cda_split_combine",
    "cda_square_layout", "cda_square_tx_share_range", "cda_square_construct", "cda_construct_extend_dah", "cda_square_construct_device",
    "cda_blob_commitments", "cda_blob_commitments_device",
    "cda_square_create", "cda_square_destroy", "cda_square_dah", "cda_square_share_proof",
    "cda_square_blob_commitments", "cda_square_subtree_root", "cda_repair", "cda_repair_device", "cda_rs_decode",
    "cda_nmt_axis_roots", "cda_nmt_axis_root", "cda_nmt_prove_range", "cda_merkle_root",
    "cda_comm_unique_id", "cda_comm_init", "cda_comm_destroy", "cda_comm_size", "cda_comm_abort", "cda_extend_dah_split", "cda_split_rows_send",
    "cda_extend_dah_multi", "cda_split_layout", "cda_split_offsets", "cda_extend_dah_batch_ex",
)
STAGES = ("rs_q0", "rs_q3", "order_check", "nmt_leaves", "nmt_levels", "data_root")


class CdaError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


class PushOrderError(CdaError):
    """nmt ErrInvalidPushOrder surfaced through RowRoots/ColRoots."""


class ByzantineDataError(CdaError):
    """rsmt2d ErrByzantineData: axis 0 (row) / 1 (col) and index of the
    first vector whose rebuilt cells contradict its root or encoding."""

    def __init__(self, rc: int, msg: str, axis: int = -1, index: int = 0):
        super().__init__(rc, msg)
        self.axis, self.index = axis, index


class UnrepairableError(CdaError):
    """rsmt2d ErrUnrepairableDataSquare / reedsolomon ErrTooFewShards."""


class SquareError(CdaError):
    """go-square square.Construct / Build error."""


class SplitLayoutT(C.Structure):
    """cda_split_layout_t (include/cda.h)."""
    _fields_ = [(n, C.c_uint32) for n in ("k", "world", "W", "R", "C")] + \
               [(n, C.c_uint64) for n in ("piece_bytes", "send_bytes", "col_block_bytes", "col_slots_off",
                                          "row_sub_off", "gather_sub_off", "gather_col_off", "err_off",
                                          "slots_bytes")]


_lib = None
_libs = {}
_lock = threading.RLock()   # re-entrant: default_context() creates a Context (load()) under it


def load(path: str | None = None):
    """Load libcda.so (or the library at `path`, e.g. TEST_LIB_PATH) and
    declare prototypes. Raises OSError if absent."""
    global _lib
    path = path or LIB_PATH
    with _lock:
        if path in _libs:
            return _libs[path]
        # One HIP runtime per process: PyTorch-ROCm bundles its own
        # libamdhip64 (same soname).  If libcda.so were loaded first, a later
        # `import torch` would map a second runtime and see no GPU; importing
        # torch first makes libcda bind to torch's copy.
        if "torch" not in sys.modules and importlib.util.find_spec("torch") is not None:
            import torch  # noqa: F401
        if not os.path.exists(path):
            raise OSError(f"{os.path.basename(path)} not built at {path}; run __graft_entry__.build() "
                          "(no CPU fallback exists)")
        L = C.CDLL(path)
        u8p = C.POINTER(C.c_uint8)
        vp = C.c_void_p
        ctxp = C.c_void_p
        L.cda_ctx_create.argtypes = [C.c_int, C.POINTER(ctxp)]
        L.cda_ctx_destroy.argtypes = [ctxp]
        L.cda_last_error.argtypes = [ctxp]
        L.cda_last_error.restype = C.c_char_p
        L.cda_version.restype = C.c_char_p
        L.cda_extend_shares.argtypes = [ctxp, u8p, C.c_uint32, u8p]
        L.cda_dah_from_eds.argtypes = [ctxp, u8p, C.c_uint32, u8p, u8p, u8p]
        L.cda_extend_dah.argtypes = [ctxp, u8p, C.c_uint32, u8p, u8p, u8p, u8p]
        L.cda_extend_dah_batch.argtypes = [ctxp, u8p, C.c_uint32, C.c_uint32, u8p, u8p, u8p, u8p,
                                           C.POINTER(C.c_int32)]
        L.cda_extend_dah_batch_ex.argtypes = [ctxp, u8p, C.c_uint32, C.c_uint32, u8p, C.c_int, u8p, u8p, u8p,
                                              C.POINTER(C.c_int32)]
        L.cda_extend_dah_device.argtypes = [ctxp, vp, C.c_uint32, C.c_uint32, vp, vp, vp, vp, vp, vp]
        L.cda_reserve.argtypes = [ctxp, C.c_uint32, C.c_uint32]
        L.cda_extend_dah_inplace_device.argtypes = [ctxp, C.c_uint32, C.c_uint32, vp, vp, vp, vp, vp, vp]
        L.cda_rs_encode.argtypes = [ctxp, u8p, C.c_uint32, C.c_uint32, C.c_uint32, u8p]
        L.cda_data_root.argtypes = [ctxp, u8p, u8p, C.c_uint32, u8p]
        L.cda_push_order_detail.argtypes = [ctxp, C.POINTER(C.c_int32), C.POINTER(C.c_uint32),
                                            C.POINTER(C.c_uint32)]
        L.cda_push_order_detail_at.argtypes = [ctxp, C.c_uint32, C.POINTER(C.c_int32), C.POINTER(C.c_uint32),
                                               C.POINTER(C.c_uint32)]
        L.cda_split_rows.argtypes = [ctxp, vp, C.c_uint32, C.c_uint32, C.c_uint32, vp, vp, vp]
        L.cda_split_cols.argtypes = [ctxp, vp, C.c_uint32, C.c_uint32, C.c_uint32, vp, vp, vp, vp]
        L.cda_split_combine.argtypes = [ctxp, vp, C.c_uint32, C.c_uint32, vp, vp, vp, vp, vp]
        u32p = C.POINTER(C.c_uint32)
        u64p = C.POINTER(C.c_uint64)
        L.cda_square_layout.argtypes = [ctxp, u8p, u64p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, u32p, u32p,
                                        u32p, u32p, C.c_uint32, u32p]
        L.cda_square_tx_share_range.argtypes = [ctxp, u8p, u64p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                                u32p, u32p, C.POINTER(C.c_int)]
        L.cda_square_construct.argtypes = [ctxp, u8p, u64p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, u8p,
                                           C.c_size_t, u32p, u32p, u32p]
        L.cda_construct_extend_dah.argtypes = [ctxp, u8p, u64p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, u8p,
                                               C.c_size_t, u8p, u8p, C.c_size_t, u8p, u32p, u32p, u32p]
        L.cda_square_construct_device.argtypes = [ctxp, u8p, u64p, C.c_uint32, vp, C.c_uint32, C.c_uint32, C.c_int,
                                                  vp, C.c_size_t, u32p, u32p, u32p, vp]
        L.cda_blob_commitments.argtypes = [ctxp, u8p, u8p, u64p, u8p, C.c_uint32, C.c_uint32, u8p]
        L.cda_blob_commitments_device.argtypes = [ctxp, u8p, u64p, u8p, C.c_uint32, C.c_uint32, vp, vp, vp]
        i32p = C.POINTER(C.c_int32)
        L.cda_square_create.argtypes = [ctxp, u8p, C.c_uint32, C.POINTER(vp)]
        L.cda_square_destroy.argtypes = [vp]
        L.cda_square_dah.argtypes = [vp, u32p, u8p, u8p, u8p, u8p]
        L.cda_square_share_proof.argtypes = [vp, C.c_uint32, C.c_uint32, u8p, u32p, u32p, i32p, i32p, u32p, u8p,
                                             u8p, u8p, u8p]
        L.cda_square_blob_commitments.argtypes = [vp, u32p, u32p, C.c_uint32, C.c_uint32, u8p]
        L.cda_square_subtree_root.argtypes = [vp, C.c_uint32, u8p, C.c_uint32, u8p]
        L.cda_repair.argtypes = [ctxp, u8p, u8p, C.c_uint32, u8p, u8p, i32p, u32p]
        L.cda_repair_device.argtypes = [ctxp, vp, u8p, C.c_uint32, u8p, u8p, i32p, u32p]
        L.cda_rs_decode.argtypes = [ctxp, u8p, u8p, C.c_uint32, C.c_uint32, C.c_uint32]
        L.cda_nmt_axis_roots.argtypes = [ctxp, u8p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, u32p, u8p, i32p]
        L.cda_nmt_axis_root.argtypes = [ctxp, u8p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, u8p]
        L.cda_nmt_prove_range.argtypes = [ctxp, u8p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                          C.c_uint32, u8p, u32p, u8p]
        L.cda_merkle_root.argtypes = [ctxp, u8p, u64p, C.c_uint32, u8p]
        L.cda_comm_unique_id.argtypes = [u8p]
        L.cda_comm_init.argtypes = [ctxp, C.c_int, C.c_int, u8p]
        L.cda_comm_destroy.argtypes = [ctxp]
        L.cda_comm_abort.argtypes = [ctxp]
        L.cda_comm_size.argtypes = [ctxp, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.cda_extend_dah_split.argtypes = [ctxp, vp, C.c_uint32, vp, vp, vp, vp, vp, vp]
        L.cda_split_rows_send.argtypes = [ctxp, vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, vp, vp, vp]
        L.cda_extend_dah_multi.argtypes = [C.POINTER(ctxp), C.c_uint32, u8p, C.c_uint32, C.c_uint32, u8p, u8p, u8p,
                                           u8p, i32p]
        L.cda_split_layout.argtypes = [C.c_uint32, C.c_uint32, C.POINTER(SplitLayoutT)]
        L.cda_split_offsets.argtypes = [C.c_uint32, C.c_uint32, C.c_int, C.c_uint32, u32p, u32p, u64p]
        L.cda_set_profiling.argtypes = [ctxp, C.c_int]
        L.cda_stage_times.argtypes = [ctxp, C.POINTER(C.c_double), C.POINTER(C.c_uint32), C.c_int]
        _libs[path] = L
        if path == LIB_PATH:
            _lib = L
        return L


def split_layout(k: int, world: int) -> dict:
    """cda_split_layout: config 5's buffer sizes and slot offsets (host only)."""
    out = SplitLayoutT()
    rc = load().cda_split_layout(k, world, C.byref(out))
    if rc != CDA_OK:
        raise CdaError(rc, f"invalid split: k={k} world={world}")
    return {n: getattr(out, n) for n, _ in SplitLayoutT._fields_}


def split_offsets(k: int, world: int, what: int, a, b=None) -> np.ndarray:
    """cda_split_offsets for arrays a, b (uint32): the split's byte offsets /
    slot indexes computed by the library's own layout functions."""
    a = np.ascontiguousarray(a, dtype=np.uint32)
    bb = None if b is None else np.ascontiguousarray(b, dtype=np.uint32)
    out = np.empty(a.size, dtype=np.uint64)
    u32p = C.POINTER(C.c_uint32)
    rc = load().cda_split_offsets(k, world, what, a.size, a.ctypes.data_as(u32p),
                                  None if bb is None else bb.ctypes.data_as(u32p),
                                  out.ctypes.data_as(C.POINTER(C.c_uint64)))
    if rc != CDA_OK:
        raise CdaError(rc, f"cda_split_offsets({k}, {world}, {what}) failed")
    return out


def ptr(a: np.ndarray | None):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "buffers must be C-contiguous"
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


class Context:
    """One libcda context (HIP device + stream)."""

    def __init__(self, device: int = -1, lib_path: str | None = None):
        self.lib = load(lib_path)
        h = C.c_void_p()
        rc = self.lib.cda_ctx_create(device, C.byref(h))
        if rc != CDA_OK:
            raise CdaError(rc, f"cda_ctx_create failed (rc={rc})")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.lib.cda_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, rc: int):
        if rc == CDA_OK:
            return
        msg = self.lib.cda_last_error(self.h).decode()
        if rc == CDA_ERR_PUSH_ORDER:
            raise PushOrderError(rc, msg)
        if rc == CDA_ERR_SQUARE:
            raise SquareError(rc, msg)
        if rc == CDA_ERR_BYZANTINE:
            raise ByzantineDataError(rc, msg)
        if rc == CDA_ERR_UNREPAIRABLE:
            raise UnrepairableError(rc, msg)
        raise CdaError(rc, msg)

    def set_profiling(self, on: bool):
        self.check(self.lib.cda_set_profiling(self.h, 1 if on else 0))

    def stage_times(self):
        """{stage: (total_ms, launches)} since the previous call."""
        ms = (C.c_double * len(STAGES))()
        n = (C.c_uint32 * len(STAGES))()
        self.check(self.lib.cda_stage_times(self.h, ms, n, len(STAGES)))
        return {s: (ms[i], n[i]) for i, s in enumerate(STAGES)}

    def extend_dah_device(self, d_ods: int, k: int, n: int, d_eds: int, d_rows: int, d_cols: int,
                          d_roots: int, d_status: int | None = None, stream: int | None = None):
        """Enqueue the whole path on device pointers (asynchronous)."""
        self.check(self.lib.cda_extend_dah_device(self.h, d_ods, k, n, d_eds, d_rows, d_cols, d_roots,
                                                  d_status, stream))

    def reserve(self, k: int, n: int):
        """Pre-size the scratch for device batches of n squares of width k."""
        self.check(self.lib.cda_reserve(self.h, k, n))

    def extend_dah_inplace_device(self, k: int, n: int, d_eds: int, d_rows: int, d_cols: int, d_roots: int,
                                  d_status: int | None = None, stream: int | None = None):
        """As extend_dah_device with the ODS already in Q0 of d_eds (asynchronous)."""
        self.check(self.lib.cda_extend_dah_inplace_device(self.h, k, n, d_eds, d_rows, d_cols, d_roots,
                                                          d_status, stream))

    # -- config 5 (one square split across ranks); device pointers as ints --
    def split_rows(self, d_rows, k, n_rows, row0, d_block, d_err, stream=None):
        self.check(self.lib.cda_split_rows(self.h, d_rows, k, n_rows, row0, d_block, d_err, stream))

    def split_cols(self, d_block, k, n_cols, col0, d_col_slots, d_row_sub, d_err, stream=None):
        self.check(self.lib.cda_split_cols(self.h, d_block, k, n_cols, col0, d_col_slots, d_row_sub, d_err, stream))

    def split_combine(self, d_row_sub, parts, k, d_col_slots, d_rows, d_cols, d_root, stream=None):
        self.check(self.lib.cda_split_combine(self.h, d_row_sub, parts, k, d_col_slots, d_rows, d_cols, d_root,
                                              stream))

    def split_rows_send(self, d_rows, k, n_rows, row0, parts, d_send, d_err, stream=None):
        """Row block of n_rows ODS rows straight in the all-to-all send layout
        [parts][R][C][512] (cda_split_rows_send)."""
        self.check(self.lib.cda_split_rows_send(self.h, d_rows, k, n_rows, row0, parts, d_send, d_err, stream))

    # -- multi-GPU inside the library (RCCL) --------------------------------
    def comm_init(self, rank: int, world: int, uid: bytes):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        self.check(self.lib.cda_comm_init(self.h, rank, world, buf))

    def comm_destroy(self):
        self.check(self.lib.cda_comm_destroy(self.h))

    def comm_size(self) -> tuple:
        """(rank, world) as the library's RCCL communicator formed them."""
        r, w = C.c_int(), C.c_int()
        self.check(self.lib.cda_comm_size(self.h, C.byref(r), C.byref(w)))
        return r.value, w.value

    def comm_abort(self):
        """ncclCommAbort (safe from a watchdog thread while a call waits)."""
        self.check(self.lib.cda_comm_abort(self.h))

    def extend_dah_split(self, d_rows, k, d_col_block, d_row_roots, d_col_roots, d_root, d_err, stream=None):
        """Config 5 on this rank with the library's own RCCL collectives."""
        self.check(self.lib.cda_extend_dah_split(self.h, d_rows, k, d_col_block, d_row_roots, d_col_roots, d_root,
                                                 d_err, stream))

    def push_order_detail(self):
        a, i, p = C.c_int32(), C.c_uint32(), C.c_uint32()
        self.lib.cda_push_order_detail(self.h, C.byref(a), C.byref(i), C.byref(p))
        return a.value, i.value, p.value

    def push_order_detail_at(self, square: int):
        """(axis, index, position) of square `square` of the last device
        batch (axis -1: ordered); waits for that batch's GPU work."""
        a, i, p = C.c_int32(), C.c_uint32(), C.c_uint32()
        self.check(self.lib.cda_push_order_detail_at(self.h, square, C.byref(a), C.byref(i), C.byref(p)))
        return a.value, i.value, p.value


def comm_unique_id() -> bytes:
    """ncclGetUniqueId (rank 0; hand the 128 bytes to every rank)."""
    L = load()
    buf = (C.c_uint8 * 128)()
    rc = L.cda_comm_unique_id(buf)
    if rc != CDA_OK:
        raise CdaError(rc, L.cda_last_error(None).decode())
    return bytes(buf)


def extend_dah_multi(ctxs, ods: np.ndarray, want_eds: bool = True):
    """Config 4 on one node: n squares (n, k*k, 512) split over the contexts
    (one per GPU), run concurrently (cda_extend_dah_multi)."""
    L = load()
    ods = np.ascontiguousarray(ods, dtype=np.uint8)
    n = ods.shape[0]
    k = int(round((ods.size // (n * SHARE_SIZE)) ** 0.5))
    W = 2 * k
    eds = np.empty((n, W, W, SHARE_SIZE), dtype=np.uint8) if want_eds else None
    rows = np.empty((n, W, NMT_ROOT_SIZE), dtype=np.uint8)
    cols = np.empty((n, W, NMT_ROOT_SIZE), dtype=np.uint8)
    roots = np.empty((n, 32), dtype=np.uint8)
    status = np.empty(n, dtype=np.int32)
    hs = (C.c_void_p * len(ctxs))(*[c.h.value for c in ctxs])
    rc = L.cda_extend_dah_multi(hs, len(ctxs), ptr(ods), k, n, ptr(eds), ptr(rows), ptr(cols), ptr(roots),
                                status.ctypes.data_as(C.POINTER(C.c_int32)))
    if rc not in (CDA_OK, CDA_ERR_PUSH_ORDER):
        ctxs[0].check(rc)
    return eds, rows, cols, roots, status


_default = None


def default_context() -> Context:
    global _default
    if _default is None:
        with _lock:
            if _default is None:
                _default = Context(int(os.environ.get("CDA_DEVICE", "-1")))
    return _default
