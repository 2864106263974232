"""Multi-GPU orchestration.

Config 4 -- a batch of independent squares: every rank extends its own
squares (`cda_extend_dah_device`), there is no data-path collective.

Config 5 -- ONE square split across G ranks (one GPU each), row blocks then
column blocks:

  1. rank g owns ODS rows [g*R, g*R+R), R = k/G: row-encode them (Q0 -> Q1)
     and check their namespace order; the row block is written straight in
     the all-to-all send layout [G][R][C] shares (cda_split_rows_send)
  2. all-to-all (RCCL over xGMI): rank g sends rank h the R x C slice of its
     row block for columns [h*C, h*C+C), C = W/G; every pair exchanges
     R*C*512 bytes (4 MiB at k=512, G=8), one point-to-point link each; the
     received pieces are rows 0..k-1 of the column block as they land (no
     host-side copies)
  3. rank h column-encodes its W x C block (Q0 -> Q2, Q1 -> Q3 -- equal to the
     reference's Q2 -> Q3 row extension by linearity), hashes every cell once,
     builds its C column roots and, for every EDS row, the NMT subtree node
     over its C columns (an aligned subtree of the row tree)
  4. gather (W + C) 96-B slots per rank on rank 0 (~100 KB per rank)
  5. rank 0 finishes the top log2(G) levels of the 2k row trees and the data
     root.

The EDS stays column-distributed (rank h holds full columns [h*C, h*C+C)).
Compute is delegated to an `ops` object: `GpuSplitOps` (libcda.so) in
production; the tests drive the same orchestration over gloo with a CPU
implementation of the three steps to check the data movement.  A host without
torch.distributed runs the same split with the library's own RCCL
communicator: `extend_dah_split_rccl` (cda_comm_init + cda_extend_dah_split).
"""
from __future__ import annotations

SHARE = 512
SLOT = 96


class GpuSplitOps:
    """The three per-rank steps on the GPU (cda_split_rows/cols/combine)."""

    def __init__(self, ctx, device):
        import torch
        self.ctx = ctx
        self.device = device
        self.torch = torch

    def _stream(self):
        return self.torch.cuda.current_stream(self.device).cuda_stream

    def new_err(self):
        return self.torch.full((1,), -1, dtype=self.torch.int32, device=self.device)

    def rows(self, ods_rows, k, row0, err):
        t = self.torch
        R = ods_rows.numel() // (k * SHARE)
        block = t.empty((R, 2 * k, SHARE), dtype=t.uint8, device=self.device)
        self.ctx.split_rows(ods_rows.data_ptr(), k, R, row0, block.data_ptr(), err.data_ptr(), self._stream())
        return block

    def rows_send(self, ods_rows, k, row0, parts, out, err):
        """Row-encode into the send layout `out` = [parts][R][C][512]."""
        R = ods_rows.numel() // (k * SHARE)
        self.ctx.split_rows_send(ods_rows.data_ptr(), k, R, row0, parts, out.data_ptr(), err.data_ptr(),
                                 self._stream())

    def cols(self, block, k, col0, err):
        t = self.torch
        W, C = block.shape[0], block.shape[1]
        col_slots = t.empty((C, SLOT), dtype=t.uint8, device=self.device)
        row_sub = t.empty((W, SLOT), dtype=t.uint8, device=self.device)
        self.ctx.split_cols(block.data_ptr(), k, C, col0, col_slots.data_ptr(), row_sub.data_ptr(),
                            err.data_ptr(), self._stream())
        return col_slots, row_sub

    def combine(self, row_sub_all, parts, k, col_slots_all):
        t = self.torch
        W = 2 * k
        rows = t.empty((W, 90), dtype=t.uint8, device=self.device)
        cols = t.empty((W, 90), dtype=t.uint8, device=self.device)
        root = t.empty((32,), dtype=t.uint8, device=self.device)
        self.ctx.split_combine(row_sub_all.data_ptr(), parts, k, col_slots_all.data_ptr(), rows.data_ptr(),
                               cols.data_ptr(), root.data_ptr(), self._stream())
        return rows, cols, root


def extend_dah_split(ods_rows, k: int, ops, rank: int, world: int, group=None, on_error=None):
    """Config 5 on this rank.  `ods_rows` = this rank's R x k ODS shares
    (tensor on the rank's device).  Returns (row_block, col_block, result)
    where result = (row_roots, col_roots, data_root, err_word) on rank 0 and
    None elsewhere.  err_word is the MIN over ranks (0xFFFFFFFF = ordered).

    on_error: if given, a failing LOCAL step calls on_error(exc) and the rank
    carries on with placeholder tensors, so every rank still enters every
    collective in the same order (a raise on one rank would leave the others
    blocked in the all-to-all or the gathers)."""
    import torch
    import torch.distributed as dist

    W = 2 * k
    if k % world or W % world:
        raise ValueError("world size must divide k")
    R, C = k // world, W // world

    def local(fn, fallback):
        if on_error is None:
            return fn()
        try:
            return fn()
        except Exception as e:  # noqa: BLE001 -- reported through on_error
            on_error(e)
            return fallback()

    err = ops.new_err()
    dev = ods_rows.device
    block = torch.empty((W, C, SHARE), dtype=torch.uint8, device=dev)       # my columns, all 2k rows
    recv = block[:k].view(world, R, C, SHARE)                                # rank g's piece = rows g*R..g*R+R-1
    send = torch.empty_like(recv) if world > 1 else recv                     # [dst][R][C][512]
    local(lambda: ops.rows_send(ods_rows, k, rank * R, world, send, err), lambda: send.zero_())
    if world > 1:
        dist.all_to_all_single(recv, send, group=group)
    col_slots, row_sub = local(lambda: ops.cols(block, k, rank * C, err),
                               lambda: (torch.zeros((C, SLOT), dtype=torch.uint8, device=dev),
                                        torch.zeros((W, SLOT), dtype=torch.uint8, device=dev)))
    err = err.to(torch.int64) & 0xFFFFFFFF          # the kernels' uint32 word; MIN needs unsigned order
    if world > 1:
        dist.all_reduce(err, op=dist.ReduceOp.MIN, group=group)
    if world > 1:
        rs = [torch.empty_like(row_sub) for _ in range(world)] if rank == 0 else None
        cs = [torch.empty_like(col_slots) for _ in range(world)] if rank == 0 else None
        dist.gather(row_sub, rs, dst=0, group=group)
        dist.gather(col_slots, cs, dst=0, group=group)
    else:
        rs, cs = [row_sub], [col_slots]
    result = None
    if rank == 0:
        row_sub_all = torch.stack(rs).contiguous()                              # [G][W][96]
        col_all = torch.cat(cs).contiguous()                                    # [W][96]
        combined = local(lambda: ops.combine(row_sub_all, world, k, col_all), lambda: None)
        result = None if combined is None else (*combined, err)
    return send, block, result


def extend_dah_split_rccl(ctx, ods_rows, k: int, rank: int, world: int, stream=None):
    """Config 5 through the library's own RCCL communicator (cda_comm_init must
    have been called on `ctx` with this rank/world): returns (col_block,
    result) with result = (row_roots, col_roots, data_root, err_word) on
    rank 0, None elsewhere."""
    import torch
    dev = ods_rows.device
    W = 2 * k
    C = W // world
    block = torch.empty((W, C, SHARE), dtype=torch.uint8, device=dev)
    err = torch.empty((1,), dtype=torch.int32, device=dev)
    rows = torch.empty((W, 90), dtype=torch.uint8, device=dev) if rank == 0 else None
    cols = torch.empty((W, 90), dtype=torch.uint8, device=dev) if rank == 0 else None
    root = torch.empty((32,), dtype=torch.uint8, device=dev) if rank == 0 else None
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    ctx.extend_dah_split(ods_rows.data_ptr(), k, block.data_ptr(), rows.data_ptr() if rank == 0 else None,
                         cols.data_ptr() if rank == 0 else None, root.data_ptr() if rank == 0 else None,
                         err.data_ptr(), stream)
    # rank 0 raises (CDA_ERR_DEVICE) when a peer failed: the reduced word is then 0
    result = (rows, cols, root, err.to(torch.int64) & 0xFFFFFFFF) if rank == 0 else None
    return block, result


def extend_dah_split_loopback(ods, k: int, parts: int, ops):
    """Config 5 with `parts` virtual ranks on ONE device (the all-to-all and
    gathers become tensor slicing): validates the split kernels and the
    subtree combine on a single GPU.  ods: (k*k, 512) tensor on the device."""
    import torch
    W = 2 * k
    R, C = k // parts, W // parts
    ods = ods.view(k, k, SHARE)
    err = ops.new_err()
    rbs = [ops.rows(ods[g * R:(g + 1) * R].contiguous(), k, g * R, err) for g in range(parts)]
    blocks, col_slots, row_subs = [], [], []
    for h in range(parts):
        block = torch.empty((W, C, SHARE), dtype=torch.uint8, device=ods.device)
        block[:k] = torch.cat([rb[:, h * C:(h + 1) * C] for rb in rbs])
        cs, rsub = ops.cols(block, k, h * C, err)
        blocks.append(block)
        col_slots.append(cs)
        row_subs.append(rsub)
    rows, cols, root = ops.combine(torch.stack(row_subs).contiguous(), parts, k, torch.cat(col_slots).contiguous())
    err = err.to(torch.int64) & 0xFFFFFFFF
    return torch.cat(blocks, dim=1), (rows, cols, root, err)
