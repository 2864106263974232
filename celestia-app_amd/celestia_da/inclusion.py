"""Mirror of go-square v1.1.0 ``inclusion`` (CreateCommitment /
CreateCommitments) over libcda.so.

Reference call sites: x/blob/types/blob_tx.go:98 (ValidateBlobTx checks every
blob's commitment against its MsgPayForBlobs) and
x/blob/types/payforblob.go:53 (NewMsgPayForBlobs), both with
merkle.HashFromByteSlices and appconsts.SubtreeRootThreshold.  All hashing
runs on the GPU in one batch (no CPU fallback).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import default_context, ptr

SUBTREE_ROOT_THRESHOLD = 64     # pkg/appconsts/v1/app_consts.go:6
NAMESPACE_SIZE = 29


@dataclass
class Blob:
    """go-square blob.Blob: namespace = version byte || 28-byte ID."""
    namespace: bytes
    data: bytes
    share_version: int = 0


def create_commitments(blobs, subtree_root_threshold: int = SUBTREE_ROOT_THRESHOLD, ctx=None):
    """inclusion.CreateCommitments: one 32-byte commitment per blob."""
    ctx = ctx or default_context()
    n = len(blobs)
    if n == 0:
        return []
    for b in blobs:
        if len(b.namespace) != NAMESPACE_SIZE:
            raise ValueError(f"namespace must be {NAMESPACE_SIZE} bytes, got {len(b.namespace)}")
    ns = np.frombuffer(b"".join(b.namespace for b in blobs), dtype=np.uint8).copy()
    off = np.zeros(n + 1, dtype=np.uint64)
    for i, b in enumerate(blobs):
        off[i + 1] = off[i] + len(b.data)
    data = np.frombuffer(b"".join(b.data for b in blobs) + b"\0", dtype=np.uint8).copy()
    ver = np.array([b.share_version & 0xFF for b in blobs], dtype=np.uint8)
    out = np.empty(n * 32, dtype=np.uint8)
    ctx.check(ctx.lib.cda_blob_commitments(ctx.h, ptr(ns), ptr(data), off.ctypes.data_as(C.POINTER(C.c_uint64)),
                                           ptr(ver), n, subtree_root_threshold, ptr(out)))
    raw = out.tobytes()
    return [raw[32 * i:32 * (i + 1)] for i in range(n)]


def create_commitment(blob: Blob, subtree_root_threshold: int = SUBTREE_ROOT_THRESHOLD, ctx=None) -> bytes:
    """inclusion.CreateCommitment."""
    return create_commitments([blob], subtree_root_threshold, ctx)[0]


def sparse_shares_needed(sequence_len: int) -> int:
    """shares.SparseSharesNeeded (first share 478 bytes, then 482)."""
    if sequence_len == 0:
        return 0
    if sequence_len < 478:
        return 1
    return 1 + -(-(sequence_len - 478) // 482)


def _round_up_pow2(x: int) -> int:
    r = 1
    while r < x:
        r <<= 1
    return r


def blob_min_square_size(share_count: int) -> int:
    """inclusion.BlobMinSquareSize."""
    s = 0
    while s * s < share_count:
        s += 1
    return _round_up_pow2(s)


def sub_tree_width(share_count: int, subtree_root_threshold: int = SUBTREE_ROOT_THRESHOLD) -> int:
    """inclusion.SubTreeWidth."""
    s = -(-share_count // subtree_root_threshold)
    return min(_round_up_pow2(s), blob_min_square_size(share_count))


def merkle_mountain_range_sizes(total: int, max_tree: int):
    """inclusion.MerkleMountainRangeSizes."""
    sizes = []
    while total:
        if total >= max_tree:
            s = max_tree
        else:
            s = 1
            while s * 2 <= total:
                s *= 2
        sizes.append(s)
        total -= s
    return sizes


def sha256_compressions(data_len: int, subtree_root_threshold: int = SUBTREE_ROOT_THRESHOLD) -> int:
    """SHA-256 compressions of one CreateCommitment: 9 per leaf (0x00 || ns ||
    share = 542 B), 3 per NMT inner node (181 B), 2 per RFC-6962 leaf (91 B)
    and inner node (65 B)."""
    n = sparse_shares_needed(data_len)
    if n == 0:
        return 0
    sizes = merkle_mountain_range_sizes(n, sub_tree_width(n, subtree_root_threshold))
    return 9 * n + 3 * sum(s - 1 for s in sizes) + 2 * len(sizes) + 2 * (len(sizes) - 1)


__all__ = ["Blob", "create_commitment", "create_commitments", "sparse_shares_needed", "sub_tree_width",
           "merkle_mountain_range_sizes", "blob_min_square_size", "sha256_compressions", "_lib"]
