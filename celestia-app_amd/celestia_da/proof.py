"""Mirror of pkg/proof (ShareProof, NewShareInclusionProofFromEDS) and
pkg/inclusion GetCommitment over a device-resident square (libcda.so).

Reference: pkg/proof/proof.go:22-206 (NewTxInclusionProof,
NewShareInclusionProof, NewShareInclusionProofFromEDS), pkg/proof/proof.pb.go (ShareProof,
RowProof, NMTProof, Proof field names), pkg/inclusion/get_commit.go:12-30.
The square is extended once (`ResidentSquare`); the EDS, every row-tree
level and the data-root tree stay in HBM, so each proof is a gather.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import NMT_ROOT_SIZE, SHARE_SIZE, default_context, ptr


@dataclass
class NMTProof:                     # proof.pb.go NMTProof
    start: int
    end: int
    nodes: list
    leaf_hash: bytes = b""


@dataclass
class Proof:                        # go-square/merkle Proof (RowProof.Proofs)
    total: int
    index: int
    leaf_hash: bytes
    aunts: list


@dataclass
class RowProof:
    row_roots: list
    proofs: list
    start_row: int
    end_row: int


@dataclass
class ShareProof:
    data: list
    share_proofs: list
    namespace_id: bytes
    row_proof: RowProof
    namespace_version: int = 0
    extra: dict = field(default_factory=dict)


def _log2(x: int) -> int:
    n = 0
    while (1 << n) < x:
        n += 1
    return n


class ResidentSquare:
    """An extended square kept on the GPU (cda_square_*)."""

    def __init__(self, ods, ctx=None):
        self.ctx = ctx or default_context()
        a = np.ascontiguousarray(np.asarray(ods, dtype=np.uint8).reshape(-1, SHARE_SIZE))
        self.h = C.c_void_p()
        rc = self.ctx.lib.cda_square_create(self.ctx.h, ptr(a), a.shape[0], C.byref(self.h))
        self.push_order_error = rc == _lib.CDA_ERR_PUSH_ORDER
        if rc not in (_lib.CDA_OK, _lib.CDA_ERR_PUSH_ORDER):
            self.ctx.check(rc)
        k = C.c_uint32()
        self.ctx.check(self.ctx.lib.cda_square_dah(self.h, C.byref(k), None, None, None, None))
        self.k = k.value

    def close(self):
        if getattr(self, "h", None):
            self.ctx.lib.cda_square_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def dah(self):
        """(row_roots, col_roots, data_root)."""
        W = 2 * self.k
        rows = np.empty(W * NMT_ROOT_SIZE, dtype=np.uint8)
        cols = np.empty(W * NMT_ROOT_SIZE, dtype=np.uint8)
        root = np.empty(32, dtype=np.uint8)
        self.ctx.check(self.ctx.lib.cda_square_dah(self.h, None, ptr(rows), ptr(cols), ptr(root), None))
        split = lambda b: [b[i * NMT_ROOT_SIZE:(i + 1) * NMT_ROOT_SIZE].tobytes() for i in range(W)]  # noqa: E731
        return split(rows), split(cols), root.tobytes()

    def eds(self) -> np.ndarray:
        W = 2 * self.k
        out = np.empty(W * W * SHARE_SIZE, dtype=np.uint8)
        self.ctx.check(self.ctx.lib.cda_square_dah(self.h, None, None, None, None, ptr(out)))
        return out.reshape(W, W, SHARE_SIZE)

    def share_proof(self, namespace: bytes, start: int, end: int) -> ShareProof:
        """proof.NewShareInclusionProofFromEDS(eds, namespace, shares.Range{start, end})."""
        k = self.k
        if not (0 <= start < end <= k * k):
            raise _lib.CdaError(_lib.CDA_ERR_INVALID, "share range out of the original square")
        W = 2 * k
        R = (end - 1) // k - start // k + 1
        M, A = 2 * _log2(W), _log2(2 * W)
        shares = np.empty((end - start) * SHARE_SIZE, dtype=np.uint8)
        ns, ne = (C.c_int32 * R)(), (C.c_int32 * R)()
        cnt = (C.c_uint32 * R)()
        nodes = np.empty(R * M * NMT_ROOT_SIZE, dtype=np.uint8)
        roots = np.empty(R * NMT_ROOT_SIZE, dtype=np.uint8)
        leaf = np.empty(R * 32, dtype=np.uint8)
        aunts = np.empty(R * A * 32, dtype=np.uint8)
        r0, r1 = C.c_uint32(), C.c_uint32()
        self.ctx.check(self.ctx.lib.cda_square_share_proof(self.h, start, end, ptr(shares), C.byref(r0), C.byref(r1),
                                                           ns, ne, cnt, ptr(nodes), ptr(roots), ptr(leaf),
                                                           ptr(aunts)))
        nb, rb, lb, ab = nodes.tobytes(), roots.tobytes(), leaf.tobytes(), aunts.tobytes()
        sp = [NMTProof(ns[i], ne[i], [nb[(i * M + q) * 90:(i * M + q + 1) * 90] for q in range(cnt[i])])
              for i in range(R)]
        proofs = [Proof(2 * W, r0.value + i, lb[32 * i:32 * (i + 1)],
                        [ab[(i * A + q) * 32:(i * A + q + 1) * 32] for q in range(A)]) for i in range(R)]
        sb = shares.tobytes()
        return ShareProof(data=[sb[i * SHARE_SIZE:(i + 1) * SHARE_SIZE] for i in range(end - start)],
                          share_proofs=sp, namespace_id=bytes(namespace[1:]),
                          row_proof=RowProof([rb[90 * i:90 * (i + 1)] for i in range(R)], proofs, r0.value, r1.value),
                          namespace_version=namespace[0])

    def blob_commitments(self, starts, share_lens, subtree_root_threshold: int = 64):
        """inclusion.GetCommitment for each (start, share_len)."""
        n = len(starts)
        s = (C.c_uint32 * max(1, n))(*starts)
        ln = (C.c_uint32 * max(1, n))(*share_lens)
        out = np.empty(32 * max(1, n), dtype=np.uint8)
        self.ctx.check(self.ctx.lib.cda_square_blob_commitments(self.h, s, ln, n, subtree_root_threshold, ptr(out)))
        b = out.tobytes()
        return [b[32 * i:32 * (i + 1)] for i in range(n)]

    def subtree_root(self, row: int, walk) -> bytes:
        """EDSSubTreeRootCacher.getSubTreeRoot (pkg/inclusion/nmt_caching.go:111-124):
        the node of EDS row tree `row` reached by `walk` (False = WalkLeft,
        True = WalkRight) from its root."""
        w = np.array([1 if x else 0 for x in walk] or [0], dtype=np.uint8)
        out = np.empty(90, dtype=np.uint8)
        self.ctx.check(self.ctx.lib.cda_square_subtree_root(self.h, row, ptr(w), len(walk), ptr(out)))
        return out.tobytes()


def _go_namespace(ns: bytes) -> str:
    """fmt %v of a go-square namespace.Namespace{Version, ID}."""
    return "{%d [%s]}" % (ns[0], " ".join(str(b) for b in ns[1:]))


def parse_namespace(raw_shares, start_share: int, end_share: int) -> bytes:
    """proof.ParseNamespace (pkg/proof/querier.go:134-166): the one namespace
    (29 bytes) of shares [start_share, end_share), with the reference's
    error texts (ValueError)."""
    if start_share < 0:
        raise ValueError(f"start share {start_share} should be positive")
    if end_share < 0:
        raise ValueError(f"end share {end_share} should be positive")
    if end_share <= start_share:
        raise ValueError(f"end share {end_share} cannot be lower or equal to the starting share {start_share}")
    if end_share > len(raw_shares):
        raise ValueError(f"end share {end_share} is higher than block shares {len(raw_shares)}")
    first = bytes(raw_shares[start_share][:29])
    for i, sh in enumerate(raw_shares[start_share:end_share]):
        ns = bytes(sh[:29])
        if ns != first:
            raise ValueError(f"shares range contain different namespaces at index {i}: "
                             f"{_go_namespace(first)} and {_go_namespace(ns)} ")
    return first


TX_NAMESPACE = b"\x00" * 28 + b"\x01"            # go-square namespace.TxNamespace
PAY_FOR_BLOB_NAMESPACE = b"\x00" * 28 + b"\x04"  # namespace.PayForBlobNamespace


def tx_share_range(txs, tx_index: int, max_square_size: int = 128, subtree_root_threshold: int = 64):
    """builder.FindTxShareRange of square.Construct's layout: (start, end,
    namespace) -- the tx namespace for a normal tx, the PFB namespace for a
    blob tx (proof.go:51-57 getTxNamespace).  Host only."""
    from .square import _flatten, _u64p
    L = _lib.load()
    buf, off = _flatten(txs)
    s, e, pfb = C.c_uint32(), C.c_uint32(), C.c_int()
    rc = L.cda_square_tx_share_range(None, ptr(buf), _u64p(off), len(txs), max_square_size, subtree_root_threshold,
                                     tx_index, C.byref(s), C.byref(e), C.byref(pfb))
    if rc != _lib.CDA_OK:
        msg = L.cda_last_error(None).decode()
        raise (_lib.SquareError if rc == _lib.CDA_ERR_SQUARE else _lib.CdaError)(rc, msg)
    return s.value, e.value, PAY_FOR_BLOB_NAMESPACE if pfb.value else TX_NAMESPACE


def new_share_inclusion_proof(ods, namespace: bytes, start: int, end: int, ctx=None) -> ShareProof:
    """NewShareInclusionProof (proof.go:59-73): extend the square, prove the
    range.  ods: the square's shares (bytes, a list of shares or an array)."""
    if isinstance(ods, (bytes, bytearray, memoryview)):
        ods = np.frombuffer(ods, dtype=np.uint8)
    elif isinstance(ods, list):
        ods = np.frombuffer(b"".join(ods), dtype=np.uint8)
    sq = ResidentSquare(ods, ctx)
    try:
        return sq.share_proof(namespace, start, end)
    finally:
        sq.close()


def new_tx_inclusion_proof(txs, tx_index: int, app_version: int = 2, ctx=None) -> ShareProof:
    """NewTxInclusionProof (proof.go:22-49): the share proof of the shares that
    hold tx tx_index of the block, in the square square.Construct builds."""
    from . import square
    if tx_index < 0:   # the Go parameter is a uint64
        raise _lib.CdaError(_lib.CDA_ERR_INVALID, f"txIndex {tx_index} is negative")
    if tx_index >= len(txs):
        raise _lib.CdaError(_lib.CDA_ERR_INVALID, f"txIndex {tx_index} out of bounds")
    ub, thr = square.SQUARE_SIZE_UPPER_BOUND, square.SUBTREE_ROOT_THRESHOLD   # appconsts, every version
    start, end, ns = tx_share_range(txs, tx_index, ub, thr)
    sq = square.construct(txs, ub, thr, ctx=ctx)
    return new_share_inclusion_proof(sq.to_bytes(), ns, start, end, ctx)


def _parse_int64(text: str) -> int:
    """strconv.ParseInt(text, 10, 64) with Go's error texts (ValueError)."""
    if not text or text.strip() != text or "_" in text:   # Go's base-10 syntax
        raise ValueError(f'strconv.ParseInt: parsing "{text}": invalid syntax')
    try:
        v = int(text, 10)
    except ValueError:
        raise ValueError(f'strconv.ParseInt: parsing "{text}": invalid syntax') from None
    if not -(1 << 63) <= v < (1 << 63):
        raise ValueError(f'strconv.ParseInt: parsing "{text}": value out of range')
    return v


def query_tx_inclusion_proof(path, txs, app_version: int = 2, ctx=None) -> ShareProof:
    """QueryTxInclusionProof's index handling (pkg/proof/querier.go:29-57) over
    a block's txs (the ABCI query's protobuf block is the caller's): path is
    the query path, [index]; errors are ValueError with the reference texts."""
    if len(path) != 1:
        raise ValueError(f"expected query path length: 1 actual: {len(path)} ")
    index = _parse_int64(path[0])
    if index < 0:
        raise ValueError(f'path[0] element: "{path[0]}" produced a negative value: {index}')
    return new_tx_inclusion_proof(txs, index, app_version, ctx)


def query_share_inclusion_proof(path, txs, app_version: int = 2, ctx=None) -> ShareProof:
    """QueryShareInclusionProof (pkg/proof/querier.go:72-128): path = [begin,
    end]; the block's square is square.Construct at the version's upper bound,
    the range must hold one namespace (ParseNamespace), then
    NewShareInclusionProof on the GPU."""
    from . import square
    if len(path) != 2:
        raise ValueError(f"expected query path length: 2 actual: {len(path)} ")
    begin, end = _parse_int64(path[0]), _parse_int64(path[1])
    sq = square.construct(txs, square.SQUARE_SIZE_UPPER_BOUND, square.SUBTREE_ROOT_THRESHOLD, ctx=ctx)
    ns = parse_namespace(sq, begin, end)
    return new_share_inclusion_proof(sq.to_bytes(), ns, begin, end, ctx)
