"""Two-stream batch pipeline (engine.hip enqueue_extend_dah): chunked RS on
one stream, NMT / data root on another, optionally on disjoint CU masks
(CDA_RS_CU).  Tuning knobs read at context creation; every setting must give
the serial path's bytes (and the serial path is pinned to the oracle by
test_gpu_parity.py)."""
import os

import numpy as np
import pytest

import coracle
from celestia_da import _lib, da

pytestmark = pytest.mark.gpu


def _ctx_with(env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return _lib.Context(int(os.environ.get("CDA_DEVICE", "-1")))
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("k,n,env", [
    (16, 6, {"CDA_PIPELINE_CHUNK": "2"}),
    (16, 6, {"CDA_PIPELINE_CHUNK": "2", "CDA_RS_CU": "8:1"}),
    (128, 3, {"CDA_PIPELINE_CHUNK": "1", "CDA_RS_CU": "16:3"}),
    (128, 3, {"CDA_PIPELINE_CHUNK": "2", "CDA_RS_CU": "8:1:1", "CDA_HASH_ALL_CUS": "1"}),
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


def test_bad_cu_split_fails_loudly():
    with pytest.raises(_lib.CdaError):
        _ctx_with({"CDA_RS_CU": "8:9"})
