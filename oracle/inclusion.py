"""Blob share commitments -- TEST INFRASTRUCTURE ONLY (oracle / checker).

Restates go-square v1.1.0 ``inclusion.CreateCommitment`` (EXT module pinned
at /root/reference/go.mod:9; not vendored), as called by the reference at
x/blob/types/blob_tx.go:98 (ValidateBlobTx) and x/blob/types/payforblob.go:53
(NewMsgPayForBlobs -> CreateCommitments) with merkle.HashFromByteSlices:

  shares   = SplitBlobs(blob)                      (sparse shares, shares.md)
  w        = SubTreeWidth(len(shares), threshold)  (data_square_layout.md)
  sizes    = MerkleMountainRangeSizes(len(shares), w)
  roots[i] = NMT root (sha256, 29-B namespaces, IgnoreMaxNamespace) of the
             leaves ns || share over the i-th run of `sizes[i]` shares
  commit   = RFC-6962 root of roots

Pinned by the share commitment of mainnet block 408's MsgPayForBlobs
(tests/test_commitments.py), i.e. by the reference's own fixture.
"""
from __future__ import annotations

import pyref
import square


def round_down_pow2(x: int) -> int:
    if x <= 0:
        raise ValueError("input must be positive")
    r = 1
    while r * 2 <= x:
        r *= 2
    return r


def merkle_mountain_range_sizes(total: int, max_tree: int):
    sizes = []
    while total:
        s = max_tree if total >= max_tree else round_down_pow2(total)
        sizes.append(s)
        total -= s
    return sizes


def create_commitment(ns: bytes, data: bytes, share_version: int = 0,
                      threshold: int = square.SUBTREE_ROOT_THRESHOLD) -> bytes:
    if share_version != 0:
        raise ValueError(f"unsupported share version: {share_version}")
    shares = square.sparse_shares(ns, data, 0) if data else []
    w = square.subtree_width(len(shares), threshold)
    roots, cur = [], 0
    for s in merkle_mountain_range_sizes(len(shares), w):
        leaves = [pyref.nmt_hash_leaf(ns + sh) for sh in shares[cur:cur + s]]
        roots.append(pyref.nmt_root_from_nodes(leaves))
        cur += s
    return pyref.merkle_root(roots)


# ------------------------------------------------- PFB decoding (fixtures)
def pfb_share_commitments(inner_tx: bytes):
    """share_commitments (field 4) of every MsgPayForBlobs in a cosmos TxRaw:
    TxRaw.body_bytes (1) -> TxBody.messages (1, Any) -> Any.value (2) where
    Any.type_url (1) == "/celestia.blob.v1.MsgPayForBlobs"."""
    out = []
    body = b""
    for fn, wt, v in square._fields(inner_tx):
        if fn == 1 and wt == 2:
            body = v
    for fn, wt, v in square._fields(body):
        if fn != 1 or wt != 2:
            continue
        url, val = b"", b""
        for afn, awt, av in square._fields(v):
            if afn == 1:
                url = av
            elif afn == 2:
                val = av
        if url == b"/celestia.blob.v1.MsgPayForBlobs":
            out.append([mv for mfn, mwt, mv in square._fields(val) if mfn == 4 and mwt == 2])
    return out
