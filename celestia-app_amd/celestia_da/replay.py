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


def _layout_k(ctx_h, lib, buf, off, n, max_square_size, threshold):
    """Square size of one flat block via cda_square_layout (host only); raises
    SquareError with go-square's message."""
    k = C.c_uint32()
    rc = lib.cda_square_layout(ctx_h, ptr(buf), _u64p(off), n, max_square_size, threshold,
                               _lib.CDA_SQUARE_CONSTRUCT, C.byref(k), None, None, None, 0, None)
    if rc != _lib.CDA_OK:
        msg = lib.cda_last_error(ctx_h).decode()
        raise (_lib.SquareError if rc == _lib.CDA_ERR_SQUARE else _lib.CdaError)(rc, msg)
    return k.value


def plan(blocks, max_square_size: int = SQUARE_SIZE_UPPER_BOUND,
         subtree_root_threshold: int = SUBTREE_ROOT_THRESHOLD):
    """Host-only layout of every block: (square sizes, errors).  A block whose
    txs go-square rejects gets size 0 and the reference's message."""
    L = _lib.load()
    sizes, errors = [], []
    for txs in blocks:
        buf, off = _flatten(txs)
        try:
            sizes.append(_layout_k(None, L, buf, off, len(txs), max_square_size, subtree_root_threshold))
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


def _stage_txs(blocks):
    """Every block's txs in ONE page-locked host buffer (one copy of the
    bytes), each block at a 16-byte aligned offset with >= 16 readable bytes
    after it (cda_square_construct_device reads whole 16-B words): (pinned
    uint8 tensor, its numpy view, [(start, tx offsets)] per block)."""
    import torch
    lay, pos = [], 0
    for txs in blocks:
        off = np.zeros(len(txs) + 1, dtype=np.uint64)
        np.cumsum(np.fromiter(map(len, txs), dtype=np.uint64, count=len(txs)), out=off[1:])
        lay.append((pos, off))
        pos += (int(off[-1]) + 16 + 15) & ~15
    pinned = torch.empty(max(pos, 16), dtype=torch.uint8, pin_memory=True)
    host = pinned.numpy()
    for txs, (start, off) in zip(blocks, lay):
        n = int(off[-1])
        if n:
            np.concatenate([np.frombuffer(t, dtype=np.uint8) for t in txs], out=host[start:start + n])
        host[start + n:start + n + 16] = 0
    return pinned, host, lay


def replay(blocks, data_hashes=None, max_square_size: int = SQUARE_SIZE_UPPER_BOUND,
           subtree_root_threshold: int = SUBTREE_ROOT_THRESHOLD, ctx=None, device=None, max_batch: int = 1024,
           max_stage_bytes: int = 1 << 31):
    """ProcessProposal's DA check for every block of `blocks` (each a list of
    tx bytes, in block order).  `data_hashes` (optional): the headers'
    DataHash per block.  Blocks of one square size go to the GPU in batches
    of at most `max_batch` squares (config 4's 1 024 at k = 128: 40 GiB of
    ODS + EDS); the blocks are staged in windows of at most `max_stage_bytes`
    of txs (page-locked host memory).  Returns one BlockResult per block."""
    import torch
    ctx = ctx or default_context()
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    blocks = list(blocks)
    out, w0, size = [], 0, 0
    for i, txs in enumerate(blocks):
        b = sum(map(len, txs)) + 32
        if i > w0 and size + b > max_stage_bytes:
            out += _replay_window(blocks[w0:i], max_square_size, subtree_root_threshold, ctx, dev, max_batch)
            w0, size = i, 0
        size += b
    out += _replay_window(blocks[w0:], max_square_size, subtree_root_threshold, ctx, dev, max_batch)
    if data_hashes is not None:
        for r, h in zip(out, data_hashes):
            r.accepted = r.error is None and r.data_root == bytes(h)
    return out


def _replay_window(blocks, max_square_size, subtree_root_threshold, ctx, dev, max_batch):
    import torch
    if not blocks:
        return []
    stream = torch.cuda.current_stream(dev).cuda_stream
    pinned, host, lay = _stage_txs(blocks)
    out = []
    for txs, (start, off) in zip(blocks, lay):
        seg = host[start:start + int(off[-1]) + 1]
        try:
            out.append(BlockResult(square_size=_layout_k(ctx.h, ctx.lib, seg, off, len(txs), max_square_size,
                                                         subtree_root_threshold)))
        except _lib.SquareError as e:
            out.append(BlockResult(error=str(e)))
    d_txs = torch.empty(pinned.numel(), dtype=torch.uint8, device=dev)
    d_txs.copy_(pinned, non_blocking=True)       # one H2D of every block's txs
    base = d_txs.data_ptr()
    batches = [(k, idx[c:c + max_batch]) for k, idx in group_by_size([r.square_size for r in out]).items()
               for c in range(0, len(idx), max_batch)]
    for k, idx in batches:
        n, W = len(idx), 2 * k
        d_ods = torch.empty((n, k * k, SHARE_SIZE), dtype=torch.uint8, device=dev)
        for j, i in enumerate(idx):
            start, off = lay[i]
            seg = host[start:start + int(off[-1]) + 1]
            kk = C.c_uint32()
            ctx.check(ctx.lib.cda_square_construct_device(
                ctx.h, ptr(seg), _u64p(off), len(blocks[i]), base + start, max_square_size,
                subtree_root_threshold, _lib.CDA_SQUARE_CONSTRUCT, d_ods[j].data_ptr(), k * k * SHARE_SIZE,
                C.byref(kk), None, None, stream))
            assert kk.value == k, (i, kk.value, k)
        d_eds = torch.empty((n, W * W * SHARE_SIZE), dtype=torch.uint8, device=dev)
        rows = torch.empty((n, W * 90), dtype=torch.uint8, device=dev)
        cols = torch.empty((n, W * 90), dtype=torch.uint8, device=dev)
        roots = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        status = torch.empty(n, dtype=torch.int32, device=dev)
        ctx.extend_dah_device(d_ods.data_ptr(), k, n, d_eds.data_ptr(), rows.data_ptr(), cols.data_ptr(),
                              roots.data_ptr(), status.data_ptr(), stream)
        st, rt = status.cpu().numpy(), roots.cpu().numpy()    # synchronises the stream
        for j, i in enumerate(idx):
            if st[j] == _lib.CDA_OK:
                out[i].data_root = rt[j].tobytes()
            else:
                out[i].error = _push_order_message(d_ods[j].cpu().numpy(), k, ctx.push_order_detail_at(j))
        del d_ods, d_eds
    torch.cuda.current_stream(dev).synchronize()   # the pinned staging outlives every read of it
    return out
