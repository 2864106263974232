"""Synthetic blocks of normal and blob transactions (host-side input generator).

Plays the role of /root/reference/test/util/blobfactory (ManyBlobTxs /
RandBlobTxs): BlobTx wire messages (go-square v1 proto, BlobTx{tx = 1;
repeated BlobProto blobs = 2; type_id = 3 = "BLOB"}, BlobProto{namespace_id =
1; data = 2; share_version = 3; namespace_version = 4}) around an opaque inner
tx.  Square construction never decodes the inner tx, so it is random bytes of
a realistic size (a signed MsgPayForBlobs is a few hundred bytes).  Normal txs
are random bytes that do not decode as a BlobTx.  Deterministic in `seed`.
"""
from __future__ import annotations

import numpy as np

NS_ID_SIZE = 28


def _varint(x: int) -> bytes:
    out = bytearray()
    while x >= 0x80:
        out.append((x & 0x7F) | 0x80)
        x >>= 7
    out.append(x)
    return bytes(out)


def _field_bytes(num: int, b: bytes) -> bytes:
    return _varint(num << 3 | 2) + _varint(len(b)) + b


def _field_varint(num: int, v: int) -> bytes:
    return _varint(num << 3) + _varint(v) if v else b""


def blob_proto(ns_id: bytes, data: bytes, share_version: int = 0, ns_version: int = 0) -> bytes:
    return (_field_bytes(1, ns_id) + (_field_bytes(2, data) if data else b"") +
            _field_varint(3, share_version) + _field_varint(4, ns_version))


def blob_tx(inner: bytes, blobs) -> bytes:
    """blobs: iterable of (ns_id (28 B), data[, share_version[, ns_version]])."""
    out = _field_bytes(1, inner) if inner else b""
    for b in blobs:
        out += _field_bytes(2, blob_proto(*b))
    return out + _field_bytes(3, b"BLOB")


def random_blob_namespace_id(rng: np.random.Generator) -> bytes:
    """Version-0 blob namespace ID: 18 zero bytes + 10 random bytes, above the
    reserved range (namespace.RandomBlobNamespace, testfactory/namespace.go)."""
    while True:
        tail = rng.integers(0, 256, 10, dtype=np.uint8).tobytes()
        if tail[:9] != b"\x00" * 9:
            return b"\x00" * 18 + tail


def normal_tx(rng: np.random.Generator, size: int) -> bytes:
    # 0x0A-led like a cosmos TxRaw (body_bytes = 1) but never type_id "BLOB"
    body = rng.integers(0, 256, max(0, size - 3), dtype=np.uint8).tobytes()
    return b"\x0a" + _varint(len(body)) + body


def random_block(seed: int, n_normal: int = 8, n_blob_txs: int = 32, blobs_per_tx=(1, 3), blob_size=(1, 20000),
                 shared_namespaces: int = 0):
    """[normal txs..., blob txs...] with random blob sizes/namespaces.
    shared_namespaces > 0 draws namespaces from a small pool (several blobs per
    namespace exercises the stable sort)."""
    rng = np.random.default_rng(seed)
    pool = [random_blob_namespace_id(rng) for _ in range(shared_namespaces)]
    txs = [normal_tx(rng, int(rng.integers(60, 600))) for _ in range(n_normal)]
    for _ in range(n_blob_txs):
        nb = int(rng.integers(blobs_per_tx[0], blobs_per_tx[1] + 1))
        blobs = []
        for _ in range(nb):
            ns = pool[int(rng.integers(0, len(pool)))] if pool else random_blob_namespace_id(rng)
            size = int(rng.integers(blob_size[0], blob_size[1] + 1))
            blobs.append((ns, rng.integers(0, 256, size, dtype=np.uint8).tobytes()))
        inner = rng.integers(0, 256, int(rng.integers(200, 400)), dtype=np.uint8).tobytes()
        txs.append(blob_tx(inner, blobs))
    return txs


def full_block_blobs(seed: int, max_square_size: int = 128, fill: float = 0.95, blob_size=(2000, 200000)):
    """(namespace_id, data) pairs filling about `fill` of max_square_size^2
    shares under the builder's worst-case accounting (shares + max padding,
    priced here as 2x shares + 1 PFB share)."""
    rng = np.random.default_rng(seed)
    budget = int(fill * max_square_size * max_square_size)
    out, used = [], 0
    while used < budget:
        size = int(rng.integers(blob_size[0], blob_size[1] + 1))
        shares = 1 + max(0, -(-(size - 478) // 482))
        if used + 2 * shares > budget:
            size = max(1, (budget - used) // 2 * 482)
            shares = 1 + max(0, -(-(size - 478) // 482))
        out.append((random_blob_namespace_id(rng), rng.integers(0, 256, size, dtype=np.uint8).tobytes()))
        used += 2 * shares + 1
    return out


def full_block(seed: int, max_square_size: int = 128, fill: float = 0.95, blob_size=(2000, 200000)):
    """One single-blob BlobTx per blob of full_block_blobs: the config-2/4-sized
    workload for the construction bench."""
    rng = np.random.default_rng(seed ^ 0x5EED)
    return [blob_tx(rng.integers(0, 256, 300, dtype=np.uint8).tobytes(), [b])
            for b in full_block_blobs(seed, max_square_size, fill, blob_size)]
