"""Mirror of the app-level DA entry points of celestia-app.

References:
  * app/extend_block.go:13-26 -- ExtendBlock(data, appVersion): square.Construct
    with the version's SquareSizeUpperBound / SubtreeRootThreshold, then
    da.ExtendShares(shares.ToBytes(square));
  * app/extend_block.go:28-32 -- IsEmptyBlock: no txs;
  * app/process_proposal.go:122-152 -- the data-availability half of
    ProcessProposal: Construct (reject on error), the proposed square size
    against the computed one, ExtendShares, NewDataAvailabilityHeader and the
    DAH hash against the header's DataHash, each rejection logged with the
    reason text reproduced here;
  * app/prepare_proposal.go:48-89 -- the data-availability half of
    PrepareProposal: square.Build over the filtered txs, ExtendShares,
    NewDataAvailabilityHeader; the block data carries the kept txs, the
    square size and the data root;
  * pkg/appconsts/versioned_consts.go:20-27 -- both versioned constants are
    v1's for every app version;
  * app/square_size.go:9-23 -- MaxEffectiveSquareSize: min(the blob module's
    GovMaxSquareSize param, SquareSizeUpperBound), DefaultGovMaxSquareSize
    (64, pkg/appconsts/initial_consts.go:10) at heights <= 1.  The proposal
    entry points take the governance value as `gov_max_square_size` (None:
    the hard bound, 128).

Each block is one GPU submission (cda_construct_extend_dah: txs -> square ->
EDS -> roots -> data root); for many blocks, celestia_da.replay batches the
squares of one size.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _lib, da, rsmt2d, square, wrapper
from ._lib import NMT_ROOT_SIZE, SHARE_SIZE, PushOrderError

LATEST_VERSION = 2   # pkg/appconsts/versioned_consts.go:9 (v2.Version)


def square_size_upper_bound(app_version: int = LATEST_VERSION) -> int:
    """appconsts.SquareSizeUpperBound (versioned_consts.go:25-27): v1's for every version."""
    return square.SQUARE_SIZE_UPPER_BOUND


def subtree_root_threshold(app_version: int = LATEST_VERSION) -> int:
    """appconsts.SubtreeRootThreshold (versioned_consts.go:20-22): v1's for every version."""
    return square.SUBTREE_ROOT_THRESHOLD


DEFAULT_GOV_MAX_SQUARE_SIZE = 64   # pkg/appconsts/initial_consts.go:10


def max_effective_square_size(gov_max_square_size: int | None = None, app_version: int = LATEST_VERSION,
                              height: int | None = None) -> int:
    """App.MaxEffectiveSquareSize (app/square_size.go:9-23)."""
    if height is not None and height <= 1:
        return DEFAULT_GOV_MAX_SQUARE_SIZE
    hard = square_size_upper_bound(app_version)
    return hard if gov_max_square_size is None else min(gov_max_square_size, hard)


def is_empty_block(txs, app_version: int = LATEST_VERSION) -> bool:
    """IsEmptyBlock (extend_block.go:30-32)."""
    return len(txs) == 0


def extend_block(txs, app_version: int = LATEST_VERSION, ctx=None) -> rsmt2d.ExtendedDataSquare:
    """ExtendBlock (extend_block.go:15-26): the block's EDS, its row / column
    roots and data root from ONE device submission; the roots seed the
    constructor's trees as da.extend_shares does.  Raises SquareError with
    go-square's message when Construct fails."""
    ub, thr = square_size_upper_bound(app_version), subtree_root_threshold(app_version)
    codec = rsmt2d.LeoRSCodec(ctx) if ctx is not None else da.default_codec()
    try:
        k, eds, rows, cols, root, _ = square.construct_extend_dah(txs, ub, thr, want_eds=True, ctx=ctx)
    except PushOrderError:   # Construct orders every namespace: not reachable from txs, kept for parity
        sq = square.construct(txs, ub, thr, ctx=ctx)
        return da.extend_shares(list(sq))
    W = 2 * k
    arr = np.frombuffer(bytearray(eds), dtype=np.uint8).reshape(W, W, SHARE_SIZE)
    r = np.frombuffer(b"".join(rows), dtype=np.uint8).reshape(W, NMT_ROOT_SIZE).copy()
    c = np.frombuffer(b"".join(cols), dtype=np.uint8).reshape(W, NMT_ROOT_SIZE).copy()
    return rsmt2d.ExtendedDataSquare(arr, codec, wrapper.new_constructor(k), roots=(r, c, root))


@dataclass
class BlockData:
    """core.Data as PrepareProposal returns it (prepare_proposal.go:84-88)."""
    txs: list
    square_size: int
    hash: bytes


def prepare_proposal_da(txs, app_version: int = LATEST_VERSION, ctx=None,
                        gov_max_square_size: int | None = None) -> BlockData:
    """PrepareProposal's DA steps (:48-89) on already filtered txs: Build
    (prioritised: normal txs, then blob txs, what fits), extend, DAH hash --
    one device submission.  The reference panics where this raises."""
    ub, thr = max_effective_square_size(gov_max_square_size, app_version), subtree_root_threshold(app_version)
    k, _, _, _, root, kept = square.construct_extend_dah(txs, ub, thr, build_mode=True, ctx=ctx)
    return BlockData([txs[i] for i in kept], k, root)


@dataclass
class ProposalVerdict:
    """ProcessProposal's DA decision for one block (:122-152)."""
    accept: bool
    reason: str | None = None     # the rejection log's reason (logInvalidPropBlock / ...Error)
    square_size: int = 0
    data_root: bytes | None = None


def _reason_square(err) -> str:
    return f"failure to compute data square from transactions: {err}"


def process_proposal_da(txs, square_size: int, data_hash: bytes, app_version: int = LATEST_VERSION,
                        ctx=None, gov_max_square_size: int | None = None) -> ProposalVerdict:
    """The data-availability checks of ProcessProposal (:122-152) for one
    block: txs, the proposer's BlockData.SquareSize and Header.DataHash."""
    ub, thr = max_effective_square_size(gov_max_square_size, app_version), subtree_root_threshold(app_version)
    try:
        k, _, _, _, root, _ = square.construct_extend_dah(txs, ub, thr, ctx=ctx)
    except _lib.SquareError as e:
        return ProposalVerdict(False, _reason_square(e))
    except PushOrderError as e:
        # the reference checks the proposed size before it extends (:133-136)
        k = square.layout(txs, ub, thr)[0]
        if k != square_size:
            return ProposalVerdict(False, _REASON_SIZE, k)
        return ProposalVerdict(False, f"failure to create new data availability header: {e}", k)
    return _verdict(k, root, square_size, data_hash)


_REASON_SIZE = "proposed square size differs from calculated square size"


def _verdict(k: int, root: bytes, square_size: int, data_hash: bytes) -> ProposalVerdict:
    if k != square_size:
        return ProposalVerdict(False, _REASON_SIZE, k)
    if root != bytes(data_hash):
        return ProposalVerdict(False, f"proposed data root {bytes(data_hash).hex().upper()} differs from "
                                      f"calculated data root {root.hex().upper()}", k, root)
    return ProposalVerdict(True, None, k, root)


def process_proposals_da(blocks, square_sizes, data_hashes, app_version: int = LATEST_VERSION, ctx=None,
                         device=None, gov_max_square_size: int | None = None) -> list[ProposalVerdict]:
    """process_proposal_da over many blocks, the squares of one size extended
    as one device batch (celestia_da.replay)."""
    from . import replay
    ub, thr = max_effective_square_size(gov_max_square_size, app_version), subtree_root_threshold(app_version)
    out = []
    for r, ss, h in zip(replay.replay(blocks, None, ub, thr, ctx=ctx, device=device), square_sizes, data_hashes):
        if r.error is not None:
            if r.square_size == 0:
                out.append(ProposalVerdict(False, _reason_square(r.error)))
            elif r.square_size != ss:   # size before the extend step's error (:133-136)
                out.append(ProposalVerdict(False, _REASON_SIZE, r.square_size))
            else:
                out.append(ProposalVerdict(False, f"failure to create new data availability header: {r.error}",
                                           r.square_size))
        else:
            out.append(_verdict(r.square_size, r.data_root, ss, h))
    return out
