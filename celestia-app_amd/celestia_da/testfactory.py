"""Synthetic random-namespace squares (host-side input generator).

Mirrors /root/reference/test/util/testfactory/common.go:36-46
(GenerateRandNamespacedRawData: random v0 blob namespace + random payload per
share, then sort all shares bytewise) with the portable PRNG of SURVEY.md 8(d):
SplitMix64, seed = 0xCE1E57A0 + square_index, bytes little-endian; per share
10 namespace-ID bytes (re-drawn while the first 9 are zero, i.e. not a blob
namespace, testfactory/namespace.go:15-28) then 483 payload bytes.
"""
from __future__ import annotations

import numpy as np

SHARE_SIZE = 512
SEED_BASE = 0xCE1E57A0
_GAMMA = np.uint64(0x9E3779B97F4A7C15)


def splitmix64_bytes(seed: int, n: int) -> np.ndarray:
    cnt = (n + 7) // 8
    with np.errstate(over="ignore"):
        z = np.uint64(seed & (2**64 - 1)) + np.arange(1, cnt + 1, dtype=np.uint64) * _GAMMA
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").view(np.uint8)[:n]


def random_namespaced_shares(count: int, square_index: int = 0) -> np.ndarray:
    """(count, 512) uint8, sorted bytewise."""
    per = 10 + 483
    stream = splitmix64_bytes(SEED_BASE + square_index, count * per + 4096)
    body = stream[: count * per].reshape(count, per)
    if np.any(~body[:, :9].any(axis=1)):          # a redraw happened: walk the stream exactly
        return _sequential(count, stream, square_index)
    out = np.zeros((count, SHARE_SIZE), dtype=np.uint8)
    out[:, 19:] = body
    return _sort_rows(out)


def _sequential(count, stream, square_index):
    need = count * 493 + 4096
    while len(stream) < need * 2:
        stream = splitmix64_bytes(SEED_BASE + square_index, need * 2)
        need *= 2
    out = np.zeros((count, SHARE_SIZE), dtype=np.uint8)
    pos = 0
    for i in range(count):
        while True:
            nid = stream[pos:pos + 10]
            pos += 10
            if nid[:9].any():
                break
        out[i, 19:29] = nid
        out[i, 29:] = stream[pos:pos + 483]
        pos += 483
    return _sort_rows(out)


def _sort_rows(a: np.ndarray) -> np.ndarray:
    v = np.ascontiguousarray(a).view(np.dtype((np.void, a.shape[1])))
    return np.sort(v, axis=0).view(np.uint8).reshape(a.shape)


def random_square(k: int, square_index: int = 0) -> np.ndarray:
    """ODS of width k as (k*k, 512), row-major."""
    return random_namespaced_shares(k * k, square_index)


def random_squares(k: int, indexes, threads: int = 0, chunk: int = 64):
    """Yield (position, (m, k*k, 512) array) chunks of random_square(k, i)
    for i in `indexes`, generated on a thread pool (numpy releases the GIL in
    the PRNG and the sort): config 4's 1 024 k = 128 squares take ~40 s on
    one core.  threads = 0: every CPU of the process's affinity, capped by
    OMP_NUM_THREADS."""
    import os
    from concurrent.futures import ThreadPoolExecutor
    idx = list(indexes)
    if threads <= 0:
        threads = len(os.sched_getaffinity(0))
        cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
        if cap > 0:
            threads = min(threads, cap)
    with ThreadPoolExecutor(max(1, threads)) as ex:
        for j0 in range(0, len(idx), chunk):
            part = list(ex.map(lambda i: random_square(k, i), idx[j0:j0 + chunk]))
            yield j0, np.stack(part)
