"""Blob share commitments (go-square inclusion.CreateCommitment), SURVEY.md
8(f) row 4.

Pin: mainnet block 408's MsgPayForBlobs carries the share commitment of its
169 275-byte blob (tests/golden/block408_txs.json.gz, from the reference
fixture x/blob/test/testdata/block_response.json); the oracle
(oracle/inclusion.py) reproduces it, and the GPU path must match both.  Other
sizes are checked against the pinned oracle (bit-exact)."""
import base64
import gzip
import hashlib
import json
import os

import numpy as np
import pytest

import inclusion as oinc
import knobs
import square as osq
from celestia_da import SquareError, blobfactory
from celestia_da import inclusion as ginc

HERE = os.path.dirname(os.path.abspath(__file__))


def block408_blobs():
    with gzip.open(os.path.join(HERE, "golden", "block408_txs.json.gz"), "rt") as f:
        d = json.load(f)
    out = []
    for t in d["txs"]:
        bt = osq.unmarshal_blob_tx(base64.b64decode(t))
        if bt is None:
            continue
        inner, blobs = bt
        commits = oinc.pfb_share_commitments(inner)[0]
        for b, c in zip(blobs, commits):
            ns = bytes([b["namespace_version"]]) + b["namespace_id"]
            out.append((ns, b["data"], c))
    return out


# sizes around the share boundaries: first share holds 478 bytes, then 482
SIZES = [1, 2, 477, 478, 479, 960, 961, 4000, 478 + 482 * 63, 478 + 482 * 63 + 1, 100_000, 1_000_000]


def random_blobs(seed, sizes):
    rng = np.random.default_rng(seed)
    return [ginc.Blob(b"\x00" + blobfactory.random_blob_namespace_id(rng), rng.integers(0, 256, s, dtype=np.uint8)
                      .tobytes()) for s in sizes]


# ------------------------------------------------------------------ CPU tests
def test_oracle_pinned_by_block408():
    blobs = block408_blobs()
    assert len(blobs) == 1 and len(blobs[0][1]) == 169275
    for ns, data, commit in blobs:
        assert oinc.create_commitment(ns, data) == commit


def test_mmr_sizes():
    # inclusion.MerkleMountainRangeSizes examples (go-square docs / ADR-013 style)
    assert oinc.merkle_mountain_range_sizes(11, 4) == [4, 4, 2, 1]
    assert oinc.merkle_mountain_range_sizes(2, 64) == [2]
    assert oinc.merkle_mountain_range_sizes(64, 8) == [8] * 8
    assert oinc.merkle_mountain_range_sizes(0, 8) == []


def test_empty_blob_commits_to_empty_hash():
    assert oinc.create_commitment(b"\x00" * 29, b"") == hashlib.sha256(b"").digest()


# ------------------------------------------------------------------ GPU tests
@pytest.mark.gpu
def test_block408_commitment_gpu(ctx):
    for ns, data, commit in block408_blobs():
        assert ginc.create_commitment(ginc.Blob(ns, data)) == commit


@pytest.mark.gpu
def test_commitments_match_oracle_gpu(ctx):
    blobs = random_blobs(5, SIZES)
    got = ginc.create_commitments(blobs)
    for b, c in zip(blobs, got):
        assert c == oinc.create_commitment(b.namespace, b.data), len(b.data)


@pytest.mark.gpu
def test_commitments_batch_many_small_gpu(ctx):
    rng = np.random.default_rng(9)
    sizes = [int(x) for x in rng.integers(1, 30_000, 300)] + [0, 0, 5]
    blobs = random_blobs(9, sizes)
    got = ginc.create_commitments(blobs)
    for b, c in zip(blobs, got):
        assert c == oinc.create_commitment(b.namespace, b.data), len(b.data)


@pytest.mark.gpu
@pytest.mark.parametrize("ucap,fused", [("1", "0"), ("100", "0"), ("1000", "0"), ("32", "1")])
def test_commitments_blob_groups_gpu(ctx, ucap, fused, monkeypatch):
    """commit.hip commitment_group_kernel with forced group sizes: one blob per
    wave (ucap 1), groups whose levels take lane pairs and single lanes, and
    groups of up to 64 blobs whose first levels take several passes of the
    wave (ucap 1000), including empty and one-share blobs; and the same
    batch through commitment_fused_kernel (subtree levels in LDS, the
    default for blobs of at most 512 shares)."""
    monkeypatch.setenv("CDA_COMMIT_UCAP", ucap)     # test knobs: read per call by the test build only
    monkeypatch.setenv("CDA_COMMIT_FUSED", fused)
    tc = knobs.ctx_with({})
    rng = np.random.default_rng(21)
    sizes = [int(x) for x in rng.integers(1, 60_000, 150)] + [0, 1, 478, 0] + [int(x) for x in rng.integers(1, 900, 40)]
    blobs = random_blobs(21, sizes)
    try:
        for threshold in (64, 2):
            got = ginc.create_commitments(blobs, threshold, ctx=tc)
            for b, c in zip(blobs, got):
                assert c == oinc.create_commitment(b.namespace, b.data, 0, threshold), (len(b.data), threshold)
    finally:
        tc.close()


@pytest.mark.gpu
def test_commitments_fused_edges_gpu(ctx):
    """commitment_fused_kernel at its limits: 512-share blobs alone in their
    group, groups up to the 384-leaf cap with alignment gaps, 64 tiny blobs
    in one group, height-0 subtrees (remainder shares), empty blobs."""
    first, cont = 478, 482
    sizes = [first + cont * 511, first + cont * 510 + 1, 0, first + cont * 200, 1, 2, first + cont * 7,
             first + cont * 2 + 5] + [1] * 70 + [first + cont * 63 + 1, 0, first + cont * 130]
    blobs = random_blobs(23, sizes)
    for threshold in (64, 8):
        got = ginc.create_commitments(blobs, threshold)
        for b, c in zip(blobs, got):
            assert c == oinc.create_commitment(b.namespace, b.data, 0, threshold), (len(b.data), threshold)


@pytest.mark.gpu
@pytest.mark.parametrize("threshold", [1, 8, 128])
def test_commitments_other_thresholds_gpu(ctx, threshold):
    blobs = random_blobs(11, [1, 500, 7000, 50_000])
    got = ginc.create_commitments(blobs, threshold)
    for b, c in zip(blobs, got):
        assert c == oinc.create_commitment(b.namespace, b.data, 0, threshold)


@pytest.mark.gpu
def test_commitment_errors_gpu(ctx):
    with pytest.raises(SquareError, match="share version"):
        ginc.create_commitment(ginc.Blob(b"\x00" * 19 + b"\x01" * 10, b"abc", 1))
    with pytest.raises(SquareError, match="namespace"):
        ginc.create_commitment(ginc.Blob(b"\x00" + b"\x01" * 28, b"abc"))


@pytest.mark.gpu
def test_commitments_device_variant(ctx):
    import ctypes as C

    import torch
    blobs = random_blobs(13, [1, 479, 30_000, 200_000])
    ns = np.frombuffer(b"".join(b.namespace for b in blobs), dtype=np.uint8).copy()
    off = np.zeros(len(blobs) + 1, dtype=np.uint64)
    for i, b in enumerate(blobs):
        off[i + 1] = off[i] + len(b.data)
    data = np.frombuffer(b"".join(b.data for b in blobs), dtype=np.uint8)
    d_data = torch.zeros(data.size + 16, dtype=torch.uint8, device="cuda")
    d_data[:data.size] = torch.from_numpy(data.copy()).cuda()
    d_out = torch.empty(32 * len(blobs), dtype=torch.uint8, device="cuda")
    ctx.check(ctx.lib.cda_blob_commitments_device(ctx.h, ginc.ptr(ns), off.ctypes.data_as(C.POINTER(C.c_uint64)),
                                                  None, len(blobs), 64, d_data.data_ptr(), d_out.data_ptr(), None))
    torch.cuda.synchronize()
    got = d_out.cpu().numpy().tobytes()
    for i, b in enumerate(blobs):
        assert got[32 * i:32 * (i + 1)] == oinc.create_commitment(b.namespace, b.data)
