"""Mirror of pkg/da (DataAvailabilityHeader, ExtendShares).

Reference: /root/reference/pkg/da/data_availability_header.go.  Function
names are the snake_case forms of the Go API; error texts are the
reference's.  All hashing and erasure coding runs in libcda.so on the GPU.
"""
from __future__ import annotations

import numpy as np

from . import _lib, rsmt2d, wrapper
from ._lib import NMT_ROOT_SIZE, SHARE_SIZE, default_context, ptr

DEFAULT_SQUARE_SIZE_UPPER_BOUND = 128   # pkg/appconsts/versioned_consts.go:25-31 (v1/v2 = 128)
MIN_SQUARE_SIZE = 1                     # pkg/appconsts/global_consts.go
MIN_SHARE_COUNT = 1
MAX_EXTENDED_SQUARE_WIDTH = DEFAULT_SQUARE_SIZE_UPPER_BOUND * 2   # data_availability_header.go:21
MIN_EXTENDED_SQUARE_WIDTH = MIN_SQUARE_SIZE * 2                    # :22
EMPTY_HASH = bytes.fromhex("e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855")


def is_power_of_two(n: int) -> bool:
    return n > 0 and (n & (n - 1)) == 0


def round_up_power_of_two(n: int) -> int:
    r = 1
    while r < n:
        r <<= 1
    return r


def square_size(n_shares: int) -> int:
    """SquareSize (:205-216)."""
    import math
    return round_up_power_of_two(int(math.ceil(math.sqrt(n_shares))))


def default_codec() -> rsmt2d.LeoRSCodec:
    """appconsts.DefaultCodec (pkg/appconsts/global_consts.go:92)."""
    return rsmt2d.new_leo_rs_codec()


def extend_shares(s) -> rsmt2d.ExtendedDataSquare:
    """ExtendShares (:65-75)."""
    n = len(s)
    if not is_power_of_two(n):
        raise ValueError(f"number of shares is not a power of 2: got {n}")
    k = square_size(n)
    return rsmt2d.compute_extended_data_square(s, default_codec(), wrapper.new_constructor(k))


class DataAvailabilityHeader:
    def __init__(self, row_roots=None, column_roots=None):
        self.row_roots = list(row_roots or [])
        self.column_roots = list(column_roots or [])
        self._hash = b""

    def hash(self) -> bytes:
        """Hash (:92-108): RFC-6962 root of rowRoots || columnRoots."""
        if self._hash:
            return self._hash
        if not self.row_roots and not self.column_roots:
            self._hash = EMPTY_HASH
            return self._hash
        w = len(self.row_roots)
        ctx = default_context()
        out = np.empty(32, dtype=np.uint8)
        items = [bytes(r) for r in self.row_roots + self.column_roots]
        if len(self.column_roots) == w and is_power_of_two(w) and all(len(r) == NMT_ROOT_SIZE for r in items):
            # the DAH of a square: 2w 90-B roots (cda_data_root's fixed layout)
            rows = np.frombuffer(b"".join(items[:w]), dtype=np.uint8).copy()
            cols = np.frombuffer(b"".join(items[w:]), dtype=np.uint8).copy()
            ctx.check(ctx.lib.cda_data_root(ctx.h, ptr(rows), ptr(cols), w, ptr(out)))
        else:
            # merkle.HashFromByteSlices over any slices (e.g. a header decoded
            # from the wire with 6 rows, or roots of another size)
            flat = np.frombuffer(b"".join(items) + b"\x00", dtype=np.uint8).copy()
            off = np.zeros(len(items) + 1, dtype=np.uint64)
            off[1:] = np.cumsum([len(x) for x in items])
            import ctypes as C
            ctx.check(ctx.lib.cda_merkle_root(ctx.h, ptr(flat), off.ctypes.data_as(C.POINTER(C.c_uint64)),
                                              len(items), ptr(out)))
        self._hash = out.tobytes()
        return self._hash

    def string(self) -> str:
        return self.hash().hex().upper()

    def equals(self, other: "DataAvailabilityHeader") -> bool:
        return self.hash() == other.hash()

    def to_proto(self) -> dict:
        """ToProto (:110-119); the message as a dict of its two fields."""
        return {"row_roots": list(self.row_roots), "column_roots": list(self.column_roots)}

    def marshal(self) -> bytes:
        """Protobuf wire bytes of celestia.core.v1.da.DataAvailabilityHeader
        (proto/celestia/core/v1/da/data_availability_header.proto:16-21:
        repeated bytes row_roots = 1; repeated bytes column_roots = 2)."""
        out = bytearray()
        for tag, roots in ((0x0A, self.row_roots), (0x12, self.column_roots)):
            for r in roots:
                out.append(tag)
                out += _uvarint(len(r))
                out += r
        return bytes(out)

    def validate_basic(self):
        """ValidateBasic (:134-162)."""
        if len(self.column_roots) < MIN_EXTENDED_SQUARE_WIDTH or len(self.row_roots) < MIN_EXTENDED_SQUARE_WIDTH:
            raise ValueError("minimum valid DataAvailabilityHeader has at least "
                             f"{MIN_EXTENDED_SQUARE_WIDTH} row and column roots")
        if len(self.column_roots) > MAX_EXTENDED_SQUARE_WIDTH or len(self.row_roots) > MAX_EXTENDED_SQUARE_WIDTH:
            raise ValueError("maximum valid DataAvailabilityHeader has at most "
                             f"{MAX_EXTENDED_SQUARE_WIDTH} row and column roots")
        if len(self.column_roots) != len(self.row_roots):
            raise ValueError(f"unequal number of row and column roots: row {len(self.row_roots)} "
                             f"col {len(self.column_roots)}")
        h = self.hash()
        if len(h) != 32:
            raise ValueError(f"wrong hash: expected size to be 32 bytes, got {len(h)} bytes")

    def is_zero(self) -> bool:
        return len(self.column_roots) == 0 or len(self.row_roots) == 0

    def square_size(self) -> int:
        return len(self.row_roots) // 2


def data_availability_header_from_proto(p: dict) -> DataAvailabilityHeader:
    """DataAvailabilityHeaderFromProto (:121-131): copy, then ValidateBasic."""
    if p is None:
        raise ValueError("nil DataAvailabilityHeader")
    d = DataAvailabilityHeader(p.get("row_roots"), p.get("column_roots"))
    d.validate_basic()
    return d


def _uvarint(n: int) -> bytes:
    out = bytearray()
    while n >= 0x80:
        out.append((n & 0x7F) | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def unmarshal_data_availability_header(buf: bytes) -> dict:
    """Parse DataAvailabilityHeader wire bytes into the to_proto() dict.
    Unknown fields are skipped as protobuf requires; malformed input raises
    ValueError (gogoproto's Unmarshal returns an error)."""
    p = {"row_roots": [], "column_roots": []}
    i, n = 0, len(buf)

    def varint():
        nonlocal i
        v, shift = 0, 0
        while True:
            if i >= n or shift > 63:
                raise ValueError("proto: unexpected EOF in varint")
            b = buf[i]
            i += 1
            v |= (b & 0x7F) << shift
            shift += 7
            if b < 0x80:
                return v

    while i < n:
        key = varint()
        field, wt = key >> 3, key & 7
        if field == 0:
            raise ValueError("proto: illegal tag 0")
        if wt == 2:
            ln = varint()
            if i + ln > n:
                raise ValueError("proto: unexpected EOF in bytes field")
            val = bytes(buf[i:i + ln])
            i += ln
            if field == 1:
                p["row_roots"].append(val)
            elif field == 2:
                p["column_roots"].append(val)
        elif field in (1, 2):
            raise ValueError(f"proto: wrong wireType = {wt} for field {field}")
        elif wt == 0:
            varint()
        elif wt == 1 or wt == 5:
            i += 8 if wt == 1 else 4
            if i > n:
                raise ValueError("proto: unexpected EOF")
        else:
            raise ValueError(f"proto: illegal wireType {wt}")
    return p


def new_data_availability_header(eds: rsmt2d.ExtendedDataSquare) -> DataAvailabilityHeader:
    """NewDataAvailabilityHeader (:44-63)."""
    rows = eds.row_roots()
    cols = eds.col_roots()
    dah = DataAvailabilityHeader(rows, cols)
    dr = eds.data_root() if hasattr(eds, "data_root") else None
    if dr is not None:
        dah._hash = dr          # memoised Hash() from the same GPU submission
    else:
        dah.hash()
    return dah


def tail_padding_share() -> bytes:
    """go-square shares.TailPaddingShares element (specs/src/specs/shares.md:71-81)."""
    ns = b"\xff" * 28 + b"\xfe"
    return ns + b"\x01" + b"\x00" * 4 + b"\x00" * (SHARE_SIZE - 29 - 5)


def min_shares():
    return [tail_padding_share()] * MIN_SHARE_COUNT


def min_data_availability_header() -> DataAvailabilityHeader:
    """MinDataAvailabilityHeader (:179-190)."""
    return new_data_availability_header(extend_shares(min_shares()))


def _batch_shape(ods: np.ndarray) -> tuple:
    """(n, k) of a batch shaped (n, k*k, 512) or (n, k, k, 512); k from the
    shape, never rounded.  n may be 0 (an empty batch: the C API
    returns CDA_OK and the outputs are empty)."""
    if ods.ndim == 4 and ods.shape[1] == ods.shape[2] and ods.shape[3] == SHARE_SIZE:
        return ods.shape[0], ods.shape[1]
    if ods.ndim == 3 and ods.shape[2] == SHARE_SIZE:
        k = int(round(ods.shape[1] ** 0.5))
        if k * k == ods.shape[1]:
            return ods.shape[0], k
    raise ValueError(f"batch must be shaped (n, k*k, {SHARE_SIZE}) or (n, k, k, {SHARE_SIZE}), got {ods.shape}")


def extend_dah_batch_parity(ods: np.ndarray, ctx=None, skip_q0: bool = False):
    """cda_extend_dah_batch_ex: the batch's roots and its parity only.

    skip_q0=False: packed parity (CDA_EDS_PARITY), (n, 3k^2, 512) -- per square
    Q1 (k rows of k shares) then EDS rows k..2k-1; skip_q0=True: the full EDS
    layout (n, 2k, 2k, 512) with Q0 left zero (CDA_EDS_SKIP_Q0).  Returns
    (parity, rows, cols, data_roots, status)."""
    ctx = ctx or default_context()
    ods = np.ascontiguousarray(ods, dtype=np.uint8)
    n, k = _batch_shape(ods)
    W = 2 * k
    if skip_q0:
        out = np.zeros((n, W, W, SHARE_SIZE), dtype=np.uint8)
        mode = _lib.CDA_EDS_SKIP_Q0
    else:
        out = np.empty((n, 3 * k * k, SHARE_SIZE), dtype=np.uint8)
        mode = _lib.CDA_EDS_PARITY
    rows = np.empty((n, W, NMT_ROOT_SIZE), dtype=np.uint8)
    cols = np.empty((n, W, NMT_ROOT_SIZE), dtype=np.uint8)
    roots = np.empty((n, 32), dtype=np.uint8)
    status = np.empty(n, dtype=np.int32)
    import ctypes as C
    rc = ctx.lib.cda_extend_dah_batch_ex(ctx.h, ptr(ods), k, n, ptr(out), mode, ptr(rows), ptr(cols), ptr(roots),
                                         status.ctypes.data_as(C.POINTER(C.c_int32)))
    if rc not in (_lib.CDA_OK, _lib.CDA_ERR_PUSH_ORDER):
        ctx.check(rc)
    return out, rows, cols, roots, status


def unpack_parity(ods: np.ndarray, par: np.ndarray) -> np.ndarray:
    """The whole EDS (W, W, 512) of one square from its ODS and its packed
    parity (extend_dah_batch_parity), as a cgo caller assembles the cells."""
    k = int(round((ods.size // SHARE_SIZE) ** 0.5))
    W = 2 * k
    eds = np.empty((W, W, SHARE_SIZE), dtype=np.uint8)
    eds[:k, :k] = ods.reshape(k, k, SHARE_SIZE)
    eds[:k, k:] = par[:k * k].reshape(k, k, SHARE_SIZE)
    eds[k:] = par[k * k:].reshape(k, W, SHARE_SIZE)
    return eds


def extend_dah_batch(ods: np.ndarray, want_eds: bool = True, ctx=None):
    """Batch of n squares (n, k*k, 512) -> (eds|None, rows, cols, data_roots, status)."""
    ctx = ctx or default_context()
    ods = np.ascontiguousarray(ods, dtype=np.uint8)
    n, k = _batch_shape(ods)
    W = 2 * k
    eds = np.empty((n, W, W, SHARE_SIZE), dtype=np.uint8) if want_eds else None
    rows = np.empty((n, W, NMT_ROOT_SIZE), dtype=np.uint8)
    cols = np.empty((n, W, NMT_ROOT_SIZE), dtype=np.uint8)
    roots = np.empty((n, 32), dtype=np.uint8)
    status = np.empty(n, dtype=np.int32)
    import ctypes as C
    rc = ctx.lib.cda_extend_dah_batch(ctx.h, ptr(ods), k, n, ptr(eds), ptr(rows), ptr(cols), ptr(roots),
                                      status.ctypes.data_as(C.POINTER(C.c_int32)))
    if rc not in (_lib.CDA_OK, _lib.CDA_ERR_PUSH_ORDER):
        ctx.check(rc)
    return eds, rows, cols, roots, status
