"""Block replay (celestia_da.replay): ProcessProposal's DA check over many
blocks (app/process_proposal.go:122-152), one device batch per square size.

CPU tests: the host planner (square sizes and go-square's rejections, the
grouping).  GPU tests: a mixed run of blocks -- mainnet block 408 (its header
DataHash), seeded synthetic blocks of several square sizes, rejected blocks --
against the per-block path (square.construct_extend_dah) and, for the small
ones, the oracle (oracle/square.py builder + coracle.extend_dah).
"""
import numpy as np
import pytest

import coracle
import square as osq
from celestia_da import blobfactory, replay
from celestia_da import square as gsq
from test_square import block408


def _bad_order_block():
    rng = np.random.default_rng(3)
    return blobfactory.random_block(12, 1, 2) + [blobfactory.normal_tx(rng, 100)]


def _blocks():
    txs408, _, h408 = block408()
    blocks = [
        txs408,                                                     # k = 32, header DataHash known
        blobfactory.random_block(1, 4, 10, (1, 2), (1, 3000)),
        _bad_order_block(),                                         # rejected by square.Construct
        blobfactory.random_block(2, 0, 40, (1, 4), (1, 40000)),
        [],                                                         # empty block: k = 1
        blobfactory.random_block(5, 30, 0),
        blobfactory.full_block(7, 64),
        blobfactory.random_block(11, 2, 80, (1, 2), (20000, 60000)),  # does not fit 32: rejected below
        blobfactory.random_block(3, 12, 25, (1, 3), (400, 30000), 3),
        blobfactory.full_block(8, 128),
    ]
    return blocks, h408


def test_group_by_size():
    assert replay.group_by_size([4, 0, 8, 4, 1, 0, 8]) == {4: [0, 3], 8: [2, 6], 1: [4]}
    assert replay.group_by_size([]) == {}


def test_plan_matches_layout_and_rejections():
    blocks, _ = _blocks()
    sizes, errors = replay.plan(blocks, 64)
    for b, k, e in zip(blocks, sizes, errors):
        if e is None:
            assert k == gsq.layout(b, 64)[0] and k > 0
        else:
            assert k == 0
    assert "normal transaction at index 3 can not be appended after blob tx" in errors[2]
    assert sizes[4] == 1
    assert errors[9] is not None and "not enough space" in errors[9]     # k = 128 block at max 64
    s32, e32 = replay.plan(blocks, 32)
    assert e32[7] is not None and "not enough space to append blob tx" in e32[7]


@pytest.mark.gpu
def test_replay_matches_per_block(ctx):
    blocks, h408 = _blocks()
    hashes = [h408] + [b"\0" * 32] * (len(blocks) - 1)
    res = replay.replay(blocks, data_hashes=hashes, ctx=ctx)
    assert len(res) == len(blocks)
    assert len({r.square_size for r in res if r.error is None}) >= 4      # several device batches
    for b, r in zip(blocks, res):
        if r.error is not None:
            assert r.square_size == 0 and r.data_root is None and r.accepted is False
            continue
        k, _, _, _, root, _ = gsq.construct_extend_dah(b, ctx=ctx)
        assert (r.square_size, r.data_root) == (k, root)
    assert res[0].data_root == h408 and res[0].accepted is True
    assert all(r.accepted is False for r in res[1:])
    assert res[2].error.startswith("normal transaction at index 3")


@pytest.mark.gpu
def test_replay_small_blocks_vs_oracle(ctx):
    blocks = [blobfactory.random_block(s, 3, 6, (1, 2), (1, 5000)) for s in range(20, 26)] + [[]]
    res = replay.replay(blocks, max_square_size=16, ctx=ctx)
    for b, r in zip(blocks, res):
        sh, ss, _, _ = osq.builder(b, 16, 64, "construct")
        ods = np.frombuffer(b"".join(sh), dtype=np.uint8).reshape(-1, 512).copy()
        assert r.error is None and r.square_size == ss
        assert r.data_root == coracle.extend_dah(ods)[3]


@pytest.mark.gpu
def test_replay_many_same_size(ctx):
    """A block-sync shaped run: 24 blocks of one size (one batch of 24)."""
    blocks = [blobfactory.full_block(100 + s, 32) for s in range(24)]
    res = replay.replay(blocks, max_square_size=32, ctx=ctx)
    assert {r.square_size for r in res} == {32}
    for b, r in zip(blocks[::5], res[::5]):
        assert r.data_root == gsq.construct_extend_dah(b, 32, ctx=ctx)[4]
    # the same blocks in batches of at most 7 squares (4 batches, the last ragged)
    chunked = replay.replay(blocks, max_square_size=32, ctx=ctx, max_batch=7)
    assert [r.data_root for r in chunked] == [r.data_root for r in res]
    # and staged in windows of about 3 blocks' txs
    window = 3 * sum(map(len, blocks[0])) + 100
    windowed = replay.replay(blocks, max_square_size=32, ctx=ctx, max_stage_bytes=window)
    assert [r.data_root for r in windowed] == [r.data_root for r in res]
