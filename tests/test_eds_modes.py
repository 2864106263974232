"""cda_extend_dah_batch_ex: the caller keeps Q0.

pkg/da/data_availability_header.go:65-75 returns an EDS whose Q0 cells are
the input shares; a cgo caller already holds them, so the library can leave
Q0 out of what it returns: CDA_EDS_SKIP_Q0 (the EDS layout, Q0 untouched) or
CDA_EDS_PARITY (per square Q1 then rows k..2k-1, packed, one linear copy per
chunk).  Both must give the full path's bytes once reassembled, on the small
serial host path and on the chunk pipeline (slot wraps, ragged tail), with
the same roots and push-order status."""
import os

import numpy as np
import pytest

import coracle
from celestia_da import CdaError, _lib, da

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


@pytest.mark.parametrize("k,n,env", [(32, 3, {}), (64, 2, {}), (32, 7, {"CDA_HOST_PIPE_CHUNK": "2"}),
                                     (16, 10, {"CDA_HOST_PIPE_CHUNK": "3"})])
def test_parity_modes_match_full_eds(ctx, k, n, env):
    ods = np.stack([coracle.random_square(k, 1200 + i) for i in range(n)])
    bad = n - 1
    sq = ods[bad].reshape(k, k, 512)
    sq[1, 2, :29], sq[1, 3, :29] = sq[1, 3, :29].copy(), sq[1, 2, :29].copy()
    full = da.extend_dah_batch(ods, ctx=ctx)
    pc = _ctx_with(env) if env else ctx
    try:
        par = da.extend_dah_batch_parity(ods, ctx=pc)
        skip = da.extend_dah_batch_parity(ods, ctx=pc, skip_q0=True)
    finally:
        if env:
            pc.close()
    for got in (par, skip):
        for a, b in zip(full[1:], got[1:]):   # rows, cols, data roots, status
            assert np.array_equal(a, b)
    assert [bool(x) for x in full[4] != 0] == [bool(x) for x in par[4] != 0]
    for i in range(n):
        assert np.array_equal(da.unpack_parity(ods[i], par[0][i]), full[0][i]), i
        assert not skip[0][i][:k, :k].any()                                     # Q0 untouched (zeros)
        assert np.array_equal(skip[0][i][:k, k:], full[0][i][:k, k:])
        assert np.array_equal(skip[0][i][k:], full[0][i][k:])
    assert bytes(full[3][0]) == coracle.extend_dah(ods[0])[3]


def test_unknown_eds_mode_rejected(ctx):
    ods = coracle.random_square(4, 0)
    out = np.empty(3 * 16 * 512, dtype=np.uint8)
    rows = np.empty(8 * 90, dtype=np.uint8)
    cols = np.empty(8 * 90, dtype=np.uint8)
    roots = np.empty(32, dtype=np.uint8)
    rc = ctx.lib.cda_extend_dah_batch_ex(ctx.h, _lib.ptr(ods), 4, 1, _lib.ptr(out), 7, _lib.ptr(rows), _lib.ptr(cols),
                                         _lib.ptr(roots), None)
    assert rc == _lib.CDA_ERR_INVALID
    with pytest.raises(CdaError, match="unknown eds_mode"):
        ctx.check(rc)


def test_parity_staging_released_with_context():
    """the packed-parity staging buffer is released when
    its context is destroyed.  Creating a context, making a CDA_EDS_PARITY
    call on the chunk pipeline and closing it, three times over, must not
    keep device memory (each round stages ~170 MiB at k=128, n=6, chunk 3)."""
    import torch
    k, n = 128, 6
    ods = np.stack([coracle.random_square(k, 1300 + i) for i in range(n)])

    def round_trip():
        pc = _ctx_with({"CDA_HOST_PIPE_CHUNK": "3"})
        try:
            da.extend_dah_batch_parity(ods, ctx=pc)
        finally:
            pc.close()

    round_trip()                       # first-use allocations (HIP runtime, pools)
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info()
    for _ in range(3):
        round_trip()
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info()
    assert free0 - free1 < 128 << 20, f"{(free0 - free1) >> 20} MiB kept after 3 context round trips"
