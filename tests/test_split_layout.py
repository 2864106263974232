"""Config 5's G > 1 exchange replayed on the CPU through the library's own
layout arithmetic.

cda_extend_dah_split (csrc/comm.hip) splits ONE square over G ranks: rank g
row-encodes ODS rows [g R, g R + R) straight into the all-to-all send layout,
the grouped ncclSend / ncclRecv all-to-all delivers rows 0..k-1 of every
rank's C columns, each rank column-encodes and hashes its columns, and rank 0
gathers the row-subtree and column-root slots and finishes the row trees and
the data root.  RCCL at G > 1 has never run on hardware here (one GPU per
box), so the offsets -- send layout, piece placement, slot area, gather
order, combine order -- are pinned on the CPU: every one of them comes from
the library (cda_split_layout / cda_split_offsets, csrc/split_layout.h, the
functions the group-rows kernel and split_extend_dah themselves use), the
collectives are plain buffer copies, and the arithmetic in between (Leopard
encode, NMT hashing) is the oracle's.  The replay must reproduce the oracle's
EDS columns, all 4k roots and the data root (pkg/da/data_availability_header.go:44-108).
Unmeasured on hardware.
"""
import numpy as np
import pytest

import coracle
import pyref
from celestia_da import _lib

SH = 512
SLOT = 96
PARITY_NS = b"\xff" * 29


def _leaf(cell: bytes, row: int, col: int, k: int) -> bytes:
    ns = cell[:29] if (row < k and col < k) else PARITY_NS
    return pyref.nmt_hash_leaf(ns + cell)


def _put_slot(buf: np.ndarray, off: int, node: bytes):
    buf[off:off + 90] = np.frombuffer(node, dtype=np.uint8)
    buf[off + 90:off + SLOT] = 0


def _get_slot(buf: np.ndarray, off: int) -> bytes:
    return buf[off:off + 90].tobytes()


def replay(k: int, G: int, seed: int):
    L = _lib.split_layout(k, G)
    W, R, C = L["W"], L["R"], L["C"]
    assert (W, R, C) == (2 * k, k // G, 2 * k // G)
    off = lambda what, a, b=None: _lib.split_offsets(k, G, what, a, b).astype(np.int64)  # noqa: E731
    ods = coracle.random_square(k, seed).reshape(k, k, SH)
    e_eds, e_rows, e_cols, e_root = coracle.extend_dah(ods.reshape(-1, SH))
    e_eds = e_eds.reshape(W, W, SH)

    # 1. each rank: its R ODS rows, row-extended, into the send layout
    rr, cc = np.meshgrid(np.arange(R), np.arange(W), indexing="ij")
    send_off = off(_lib.CDA_SPLIT_SEND, rr.ravel(), cc.ravel())
    assert len(set(send_off.tolist())) == R * W and send_off.max() + SH <= L["send_bytes"]
    send = []
    for g in range(G):
        rows = ods[g * R:(g + 1) * R]
        block = np.concatenate([rows, np.stack([coracle.leopard_encode(r) for r in rows])], axis=1)   # [R][W]
        buf = np.zeros(L["send_bytes"], dtype=np.uint8)
        for i, o in enumerate(send_off):
            buf[o:o + SH] = block[rr.ravel()[i], cc.ravel()[i]]
        send.append(buf)

    # 2. all-to-all: rank g's piece h -> rank h, landing where rank g's piece goes
    piece = L["piece_bytes"]
    sp = off(_lib.CDA_SPLIT_SEND_PIECE, np.arange(G))
    rp = off(_lib.CDA_SPLIT_RECV_PIECE, np.arange(G))
    blocks = []
    for h in range(G):
        blk = np.zeros(L["col_block_bytes"], dtype=np.uint8)
        for g in range(G):
            blk[rp[g]:rp[g] + piece] = send[g][sp[h]:sp[h] + piece]
        blocks.append(blk)

    # 3. each rank: its C columns (rows 0..k-1 arrived; rows k..W-1 encoded),
    #    column roots and one row-subtree node per EDS row
    br, bc = np.meshgrid(np.arange(W), np.arange(C), indexing="ij")
    boff = off(_lib.CDA_SPLIT_BLOCK, br.ravel(), bc.ravel()).reshape(W, C)
    slots = []
    for h in range(G):
        blk = blocks[h]
        cell = lambda r, c: blk[boff[r, c]:boff[r, c] + SH]  # noqa: E731
        for c in range(C):   # the exchange delivered the oracle's rows 0..k-1 of column h C + c
            for r in range(k):
                assert np.array_equal(cell(r, c), e_eds[r, h * C + c]), (h, r, c)
            data = np.stack([cell(r, c) for r in range(k)])
            par = coracle.leopard_encode(data)
            for i in range(k):
                blk[boff[k + i, c]:boff[k + i, c] + SH] = par[i]
        got = np.stack([np.stack([cell(r, c) for c in range(C)]) for r in range(W)])
        assert np.array_equal(got, e_eds[:, h * C:(h + 1) * C]), h
        leaves = [[_leaf(bytes(got[r, c]), r, h * C + c, k) for c in range(C)] for r in range(W)]
        sl = np.zeros(L["slots_bytes"], dtype=np.uint8)
        for c in range(C):
            _put_slot(sl, L["col_slots_off"] + c * SLOT, pyref.nmt_root_from_nodes([leaves[r][c] for r in range(W)]))
        for r in range(W):
            _put_slot(sl, L["row_sub_off"] + r * SLOT, pyref.nmt_root_from_nodes(leaves[r]))
        slots.append(sl)

    # 4. gather on rank 0 (rank order), as the library's grouped receives place them
    gs = off(_lib.CDA_SPLIT_GATHER_SUB, np.arange(G))
    gc = off(_lib.CDA_SPLIT_GATHER_COL, np.arange(G))
    assert gs[0] == L["gather_sub_off"] and gc[0] == L["gather_col_off"]
    s0 = slots[0]
    for h in range(G):
        s0[gs[h]:gs[h] + W * SLOT] = slots[h][L["row_sub_off"]:L["row_sub_off"] + W * SLOT]
        s0[gc[h]:gc[h] + C * SLOT] = slots[h][L["col_slots_off"]:L["col_slots_off"] + C * SLOT]
    assert gc[G - 1] + C * SLOT <= L["err_off"] < L["slots_bytes"]

    # 5. rank 0: row tree r from the G subtree nodes (combine order), column roots in rank order
    gg, rw = np.meshgrid(np.arange(G), np.arange(W), indexing="ij")
    comb = off(_lib.CDA_SPLIT_COMBINE, gg.ravel(), rw.ravel()).reshape(G, W)
    rows = [pyref.nmt_root_from_nodes([_get_slot(s0, L["gather_sub_off"] + comb[g, r] * SLOT) for g in range(G)])
            for r in range(W)]
    cols = [_get_slot(s0, L["gather_col_off"] + j * SLOT) for j in range(W)]
    return rows, cols, pyref.merkle_root(rows + cols), (e_rows, e_cols, e_root)


@pytest.mark.parametrize("k,G", [(16, 1), (16, 2), (16, 4), (16, 8), (16, 16), (32, 8)])
def test_split_exchange_replay_matches_oracle(k, G):
    rows, cols, root, (e_rows, e_cols, e_root) = replay(k, G, seed=40 + G)
    assert rows == [bytes(r) for r in e_rows]
    assert cols == [bytes(c) for c in e_cols]
    assert root == e_root


def test_split_layout_rejects_bad_shapes():
    for k, G in ((12, 2), (16, 3), (8, 16), (2048, 2), (16, 0)):
        with pytest.raises(_lib.CdaError):
            _lib.split_layout(k, G)


def test_split_layout_sizes():
    L = _lib.split_layout(512, 8)
    assert (L["R"], L["C"]) == (64, 128)
    assert L["piece_bytes"] == 64 * 128 * SH == 4 << 20            # 4 MiB per rank pair
    assert L["send_bytes"] == 8 * L["piece_bytes"] == 32 << 20     # 32 MiB send, 64 MiB column block
    assert L["col_block_bytes"] == 1024 * 128 * SH == 64 << 20


def test_split_offsets_reject_out_of_range():
    k, G = 16, 4                       # R = 4, C = 8, W = 32
    ok = _lib.split_offsets(k, G, _lib.CDA_SPLIT_SEND, [3], [31])
    assert ok[0] == ((3 * 4 + 3) * 8 + 7) * SH          # col 31: piece 3, local column 7
    for what, a, b in ((_lib.CDA_SPLIT_SEND, [4], [0]),            # r >= R
                       (_lib.CDA_SPLIT_SEND, [0], [32]),           # col >= W
                       (_lib.CDA_SPLIT_SEND, [0], None),           # b needed
                       (_lib.CDA_SPLIT_BLOCK, [32], [0]),          # row >= W
                       (_lib.CDA_SPLIT_BLOCK, [0], [8]),           # c >= C
                       (_lib.CDA_SPLIT_COMBINE, [4], [0]),         # rank >= G
                       (_lib.CDA_SPLIT_SEND_PIECE, [4], None),
                       (_lib.CDA_SPLIT_GATHER_COL, [7], None),
                       (99, [0], [0])):                            # unknown kind
        with pytest.raises(_lib.CdaError):
            _lib.split_offsets(k, G, what, a, b)
