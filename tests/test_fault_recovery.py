"""A failed call must leave the context usable.

ProcessProposal rejects a block on any error and the node keeps running
(reference: app/process_proposal.go:29-35 recovers, :138-147 rejects), so an
error return half-way through a call -- after GPU work was queued on the
context's side streams -- must not leave that work unordered before the next
call.  CDA_FAULT (tests only, read at context creation, fires once) injects an
error at three such points:

  * dah_part     -- enqueue_dah's second hash part (aux stream), after its
                    leaves, levels and data roots were queued;
  * extend_chunk -- the RS chunk pipeline (CDA_PIPELINE_CHUNK), after chunk 0's
                    RS was queued on the aux stream;
  * pipe_chunk   -- the host-buffer chunk pipeline (CDA_HOST_PIPE_CHUNK),
                    after chunk 1's H2D / compute / D2H were queued on three
                    streams.

Each test checks the injected error text, then makes follow-up calls on the
same context that grow its scratch (bigger batches: the old buffers are freed
in stream order while the failed call's side-stream work would still read
them if it were not joined) and compares every data root with the oracle.
Also the host pipeline itself: slot reuse, a ragged last
chunk, eds=NULL and a push-order violation in a late chunk, byte for byte
against the serial path.
"""
import os

import numpy as np
import pytest

import coracle
from celestia_da import CdaError, _lib, da
import knobs

pytestmark = pytest.mark.gpu


def _ctx_with(env):
    return knobs.ctx_with(env)   # CDA_FAULT is read only by the test build (csrc/knobs.h)


def _squares(k, n, seed):
    return np.stack([coracle.random_square(k, seed + i) for i in range(n)])


def _oracle_roots(ods):
    return [coracle.extend_dah(o)[3] for o in ods]


def test_dah_part_fault_host_then_clean_calls():
    pc = _ctx_with({"CDA_FAULT": "dah_part"})
    try:
        ods = _squares(32, 4, 500)
        with pytest.raises(CdaError, match="CDA_FAULT=dah_part"):
            da.extend_dah_batch(ods, ctx=pc)
        # larger batches: leaf / level slots, digests and staging all grow
        for k, n, seed in ((64, 6, 510), (32, 4, 500), (128, 3, 520)):
            ods = _squares(k, n, seed)
            eds, rows, cols, roots, status = da.extend_dah_batch(ods, ctx=pc)
            assert list(status) == [0] * n
            assert [bytes(r) for r in roots] == _oracle_roots(ods)
            e_eds = coracle.extend_dah(ods[-1])[0]
            assert np.array_equal(eds[-1].reshape(-1, 512), e_eds)
    finally:
        pc.close()


def test_dah_part_fault_device_then_clean_calls():
    import torch
    pc = _ctx_with({"CDA_FAULT": "dah_part"})
    try:
        def run(k, n, seed):
            ods = _squares(k, n, seed)
            W = 2 * k
            d_eds = torch.zeros((n, W, W, 512), dtype=torch.uint8, device="cuda")
            d_eds[:, :k, :k] = torch.from_numpy(ods.reshape(n, k, k, 512)).to("cuda")
            d_rows = torch.empty((n, W, 90), dtype=torch.uint8, device="cuda")
            d_cols = torch.empty_like(d_rows)
            d_roots = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
            pc.extend_dah_inplace_device(k, n, d_eds.data_ptr(), d_rows.data_ptr(), d_cols.data_ptr(),
                                         d_roots.data_ptr())
            torch.cuda.synchronize()
            return ods, d_roots.cpu().numpy()
        with pytest.raises(CdaError, match="CDA_FAULT=dah_part"):
            run(32, 8, 600)
        for k, n, seed in ((64, 12, 610), (128, 4, 620)):
            ods, roots = run(k, n, seed)
            assert [bytes(r) for r in roots] == _oracle_roots(ods)
    finally:
        pc.close()


def test_extend_chunk_fault_then_clean_calls():
    import torch
    pc = _ctx_with({"CDA_FAULT": "extend_chunk", "CDA_PIPELINE_CHUNK": "2"})
    try:
        def run(k, n, seed):
            ods = _squares(k, n, seed)
            W = 2 * k
            d_ods = torch.from_numpy(ods.reshape(-1)).to("cuda")
            d_eds = torch.empty((n, W, W, 512), dtype=torch.uint8, device="cuda")
            d_rows = torch.empty((n, W, 90), dtype=torch.uint8, device="cuda")
            d_cols = torch.empty_like(d_rows)
            d_roots = torch.empty((n, 32), dtype=torch.uint8, device="cuda")
            pc.extend_dah_device(d_ods.data_ptr(), k, n, d_eds.data_ptr(), d_rows.data_ptr(), d_cols.data_ptr(),
                                 d_roots.data_ptr())
            torch.cuda.synchronize()
            return ods, d_roots.cpu().numpy()
        with pytest.raises(CdaError, match="CDA_FAULT=extend_chunk"):
            run(64, 5, 700)
        for k, n, seed in ((64, 5, 700), (128, 6, 710)):
            ods, roots = run(k, n, seed)
            assert [bytes(r) for r in roots] == _oracle_roots(ods)
    finally:
        pc.close()


def test_pipe_chunk_fault_then_clean_calls(ctx):
    pc = _ctx_with({"CDA_FAULT": "pipe_chunk", "CDA_HOST_PIPE_CHUNK": "2"})
    try:
        ods = _squares(32, 7, 800)
        with pytest.raises(CdaError, match="CDA_FAULT=pipe_chunk"):
            da.extend_dah_batch(ods, ctx=pc)
        ref = da.extend_dah_batch(ods, ctx=ctx)
        got = da.extend_dah_batch(ods, ctx=pc)
        for a, b in zip(ref, got):
            assert np.array_equal(a, b)
        ods = _squares(64, 9, 810)   # bigger slots: the ring's buffers grow
        eds, rows, cols, roots, status = da.extend_dah_batch(ods, ctx=pc)
        assert [bytes(r) for r in roots] == _oracle_roots(ods)
    finally:
        pc.close()


@pytest.mark.parametrize("chunk,n", [(1, 7), (2, 7), (3, 11)])
def test_host_pipeline_matches_serial(ctx, chunk, n):
    """Engine::host_pipeline (n > 2 chunks): slot wraps (i >= 3), a ragged last
    chunk, eds=NULL, and a namespace-order violation in a late chunk, byte for
    byte against the context's serial host path and the oracle."""
    k = 32
    ods = _squares(k, n, 900 + chunk)
    bad = n - 2                      # in the last or second-to-last chunk
    sq = ods[bad].reshape(k, k, 512)
    sq[4, 9, :29], sq[4, 10, :29] = sq[4, 10, :29].copy(), sq[4, 9, :29].copy()
    if bytes(sq[4, 9, :29]) == bytes(sq[4, 10, :29]):
        pytest.skip("equal namespaces")
    pc = _ctx_with({"CDA_HOST_PIPE_CHUNK": str(chunk)})
    try:
        ref = da.extend_dah_batch(ods, ctx=ctx)          # serial host path (n <= 2 default chunks)
        got = da.extend_dah_batch(ods, ctx=pc)
        for a, b in zip(ref, got):
            assert np.array_equal(a, b)
        assert [bool(x) for x in got[4] != 0] == [i == bad for i in range(n)]
        ok = [i for i in range(n) if i != bad]
        assert [bytes(got[3][i]) for i in ok] == _oracle_roots(ods[ok])
        e_eds = coracle.extend_dah(ods[-1])[0]
        assert np.array_equal(got[0][-1].reshape(-1, 512), e_eds)
        no_eds = da.extend_dah_batch(ods, want_eds=False, ctx=pc)
        assert no_eds[0] is None
        for a, b in zip(ref[1:], no_eds[1:]):
            assert np.array_equal(a, b)
    finally:
        pc.close()
