"""Block replay: ProcessProposal's data-availability check over many blocks.

Reference: app/process_proposal.go:122-152.  Per block the proposal handler
runs square.Construct(txs, maxSquareSize, subtreeRootThreshold) (:122-126;
an error rejects the block), da.ExtendShares (:138), da.NewDataAvailabilityHeader
(:144; an error -- e.g. nmt ErrInvalidPushOrder -- rejects it) and compares
the DAH hash with the header's DataHash (:148-152).  A node that re-validates
many blocks (state sync, replay, an archival indexer) runs that loop block
after block.

Here the squares of every block are written on the GPU (the layout is planned
on the host, cda_square_construct_device) into one ODS batch per square size,
and each batch is extended and hashed as ONE device submission
(cda_extend_dah_device) -- config 4's shape (BASELINE.json configs[3], "batch
of independent squares ... block-sync replay").  Per block the result holds
what ProcessProposal decides on: the square size, the data root, and the
error that would reject it (go-square's message, or the nmt push-order
message rebuilt from cda_push_order_detail_at), plus `accepted` when the
expected data hashes are given.

This module is host plumbing over the C ABI (device buffers via torch); the
Go equivalent is the same loop over the cgo entry points.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import SHARE_SIZE, default_context, ptr
from .square import SQUARE_SIZE_UPPER_BOUND, SUBTREE_ROOT_THRESHOLD, _flatten, _u64p


@dataclass
class BlockResult:
    """One block's data-availability outcome (ProcessProposal :122-152)."""
    square_size: int = 0
    data_root: bytes | None = None
    error: str | None = None          # the message ProcessProposal would reject with
    accepted: bool | None = None      # data_root == expected DataHash (when given)


def plan(blocks, max_square_size: int = SQUARE_SIZE_UPPER_BOUND,
         subtree_root_threshold: int = SUBTREE_ROOT_THRESHOLD):
    """Host-only layout of every block: (square sizes, errors).  A block whose
    txs go-square rejects gets size 0 and the reference's message."""
    from .square import layout
    sizes, errors = [], []
    for txs in blocks:
        try:
            k, _, _ = layout(txs, max_square_size, subtree_root_threshold)
            sizes.append(k)
            errors.append(None)
        except _lib.SquareError as e:
            sizes.append(0)
            errors.append(str(e))
    return sizes, errors


def group_by_size(sizes):
    """{k: [block indexes]} in block order, failed blocks (k = 0) left out."""
    groups: dict[int, list[int]] = {}
    for i, k in enumerate(sizes):
        if k:
            groups.setdefault(k, []).append(i)
    return groups


def _push_order_message(ods_sq: np.ndarray, k: int, detail) -> str:
    axis, index, pos = detail
    cells = ods_sq.reshape(k, k, SHARE_SIZE)

    def cell(p):
        return cells[index, p] if axis == 0 else cells[p, index]
    return ("pushed data has to be lexicographically ordered by namespace IDs: last namespace: "
            f"{bytes(cell(pos - 1)[:29]).hex()}, pushed: {bytes(cell(pos)[:29]).hex()}")


def replay(blocks, data_hashes=None, max_square_size: int = SQUARE_SIZE_UPPER_BOUND,
           subtree_root_threshold: int = SUBTREE_ROOT_THRESHOLD, ctx=None, device=None):
    """ProcessProposal's DA check for every block of `blocks` (each a list of
    tx bytes, in block order).  `data_hashes` (optional): the headers'
    DataHash per block.  Returns one BlockResult per block."""
    import torch
    ctx = ctx or default_context()
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    stream = torch.cuda.current_stream(dev).cuda_stream
    sizes, errors = plan(blocks, max_square_size, subtree_root_threshold)
    out = [BlockResult(square_size=k, error=e) for k, e in zip(sizes, errors)]
    for k, idx in group_by_size(sizes).items():
        n, W = len(idx), 2 * k
        d_ods = torch.empty((n, k * k, SHARE_SIZE), dtype=torch.uint8, device=dev)
        for j, i in enumerate(idx):
            buf, off = _flatten(blocks[i])
            d_txs = torch.zeros(buf.size + 16, dtype=torch.uint8, device=dev)   # >= 16 B readable slack
            d_txs[:buf.size].copy_(torch.from_numpy(buf))
            kk = C.c_uint32()
            kept = (C.c_uint32 * max(1, len(blocks[i])))()
            n_kept = C.c_uint32()
            ctx.check(ctx.lib.cda_square_construct_device(
                ctx.h, ptr(buf), _u64p(off), len(blocks[i]), d_txs.data_ptr(), max_square_size,
                subtree_root_threshold, _lib.CDA_SQUARE_CONSTRUCT, d_ods[j].data_ptr(), k * k * SHARE_SIZE,
                C.byref(kk), kept, C.byref(n_kept), stream))
            assert kk.value == k, (i, kk.value, k)
        d_eds = torch.empty((n, W * W * SHARE_SIZE), dtype=torch.uint8, device=dev)
        rows = torch.empty((n, W * 90), dtype=torch.uint8, device=dev)
        cols = torch.empty((n, W * 90), dtype=torch.uint8, device=dev)
        roots = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        status = torch.empty(n, dtype=torch.int32, device=dev)
        ctx.extend_dah_device(d_ods.data_ptr(), k, n, d_eds.data_ptr(), rows.data_ptr(), cols.data_ptr(),
                              roots.data_ptr(), status.data_ptr(), stream)
        torch.cuda.synchronize(dev)
        st, rt = status.cpu().numpy(), roots.cpu().numpy()
        for j, i in enumerate(idx):
            if st[j] == _lib.CDA_OK:
                out[i].data_root = rt[j].tobytes()
            else:
                out[i].error = _push_order_message(d_ods[j].cpu().numpy(), k, ctx.push_order_detail_at(j))
        del d_ods, d_eds
    if data_hashes is not None:
        for r, h in zip(out, data_hashes):
            r.accepted = r.error is None and r.data_root == bytes(h)
    return out
