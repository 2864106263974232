"""Batch pipeline (engine.hip enqueue_extend_dah): each chunk's RS on an
internal stream, its leaves and wide NMT levels on the caller's stream after
an event, and the narrow levels, tree tops and data roots once for the whole
batch (dah_finish).  Tuning knobs are read at context creation; every setting
must give the serial path's bytes (and the serial path is pinned to the oracle
by test_gpu_parity.py)."""
import os

import numpy as np
import pytest

import coracle
from celestia_da import _lib, da
import knobs

pytestmark = pytest.mark.gpu


def _ctx_with(env):
    return knobs.ctx_with(env)   # A/B schedule knobs: the test build reads them (csrc/knobs.h)


@pytest.mark.parametrize("k,n,env", [
    (16, 6, {"CDA_PIPELINE_CHUNK": "2"}),
    (16, 5, {"CDA_PIPELINE_CHUNK": "2"}),                     # ragged last chunk
    (128, 3, {"CDA_PIPELINE_CHUNK": "1"}),
    (128, 6, {"CDA_PIPELINE_CHUNK": "4"}),                    # 4 + 2
    (128, 4, {"CDA_PIPELINE_CHUNK": "2", "CDA_RS8_LDS": "98304"}),
    (128, 4, {"CDA_PIPELINE_CHUNK": "2", "CDA_RS_PRIORITY": "-1"}),
    (64, 8, {"CDA_PIPELINE_CHUNK": "3"}),
])
def test_pipeline_matches_serial(ctx, k, n, env):
    ods = np.stack([coracle.random_square(k, i) for i in range(n)])
    ref = da.extend_dah_batch(ods, ctx=ctx)
    pc = _ctx_with(env)
    try:
        got = da.extend_dah_batch(ods, ctx=pc)
    finally:
        pc.close()
    for a, b in zip(ref, got):
        assert np.array_equal(a, b)
    e_eds, e_rows, e_cols, e_root = coracle.extend_dah(ods[-1])
    assert bytes(got[3][-1]) == e_root


def test_pipeline_push_order_status_per_square():
    """A namespace-order violation in one square of a later chunk is reported
    for that square only (the push-order words are filled once per batch and
    the status written by the batch's data-root launch)."""
    k, n = 32, 5
    ods = np.stack([coracle.random_square(k, i) for i in range(n)])
    bad = ods[3].reshape(k, k, 512)
    bad[2, 5, :29], bad[2, 6, :29] = bad[2, 6, :29].copy(), bad[2, 5, :29].copy()
    if bytes(bad[2, 5, :29]) == bytes(bad[2, 6, :29]):
        pytest.skip("equal namespaces")
    pc = _ctx_with({"CDA_PIPELINE_CHUNK": "2"})
    try:
        _, _, _, roots, status = da.extend_dah_batch(ods, ctx=pc)
        ref = da.extend_dah_batch(ods, ctx=None)
    finally:
        pc.close()
    assert list(status != 0) == [False, False, False, True, False]
    assert np.array_equal(roots[[0, 1, 2, 4]], ref[3][[0, 1, 2, 4]])


@pytest.mark.parametrize("k,n", [(128, 2), (128, 5), (64, 3), (16, 4), (2, 2), (1, 3), (256, 2)])
def test_hash_split_matches_one_stream(ctx, k, n):
    """The default schedule hashes a batch's two halves on two streams, each
    finishing its own trees (fused tree top for small batches) and data roots;
    CDA_HASH_SPLIT=0 is the one-stream schedule.  Same bytes, and the last
    square's data root equals the oracle's."""
    ods = np.stack([coracle.random_square(k, 100 + i) for i in range(n)])
    got = da.extend_dah_batch(ods, ctx=ctx)
    pc = _ctx_with({"CDA_HASH_SPLIT": "0"})
    try:
        ref = da.extend_dah_batch(ods, ctx=pc)
    finally:
        pc.close()
    for a, b in zip(ref, got):
        assert np.array_equal(a, b)
    assert bytes(got[3][-1]) == coracle.extend_dah(ods[-1])[3]
    assert bytes(got[3][0]) == coracle.extend_dah(ods[0])[3]


@pytest.mark.parametrize("bad", [0, 3])
def test_hash_split_push_order_status(ctx, bad):
    """Default schedule (two-part hash split; the first RS launch sets the
    push-order words): a namespace-order violation in square `bad` -- in the
    part on the caller's stream (0) or on the second stream (3) -- sets that
    square's status only; the other data roots equal the oracle's."""
    k, n = 32, 4
    ods = np.stack([coracle.random_square(k, 200 + i) for i in range(n)])
    sq = ods[bad].reshape(k, k, 512)
    sq[3, 7, :29], sq[3, 8, :29] = sq[3, 8, :29].copy(), sq[3, 7, :29].copy()
    if bytes(sq[3, 7, :29]) == bytes(sq[3, 8, :29]):
        pytest.skip("equal namespaces")
    _, _, _, roots, status = da.extend_dah_batch(ods, ctx=ctx)
    assert [bool(x) for x in status != 0] == [i == bad for i in range(n)]
    for i in range(n):
        if i != bad:
            assert bytes(roots[i]) == coracle.extend_dah(ods[i])[3]
