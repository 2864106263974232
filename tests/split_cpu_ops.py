"""CPU implementation of the three config-5 steps for the gloo tests of
celestia_da.dist (TEST INFRASTRUCTURE: oracle arithmetic; the product runs
GpuSplitOps on libcda.so)."""
import numpy as np
import torch

import pyref

SHARE, SLOT = 512, 96
NS = 29


def _ns(cell: bytes, quadrant0: bool) -> bytes:
    return cell[:NS] if quadrant0 else pyref.PARITY_NS


class CpuSplitOps:
    def new_err(self):
        return torch.full((1,), -1, dtype=torch.int32)

    @staticmethod
    def _lower(err, key):
        cur = int(err.item()) & 0xFFFFFFFF
        if key < cur:
            err.fill_(key if key < 2**31 else key - 2**32)

    def rows(self, ods_rows, k, row0, err):
        a = ods_rows.numpy().reshape(-1, k, SHARE)
        R = a.shape[0]
        out = np.empty((R, 2 * k, SHARE), dtype=np.uint8)
        for r in range(R):
            out[r, :k] = a[r]
            out[r, k:] = pyref.leopard_encode(a[r])
            for c in range(k - 1):
                if bytes(a[r, c + 1, :NS]) < bytes(a[r, c, :NS]):
                    self._lower(err, (0 << 24) | ((row0 + r) << 12) | (c + 1))
        return torch.from_numpy(out)

    def rows_send(self, ods_rows, k, row0, parts, out, err):
        rb = self.rows(ods_rows, k, row0, err)                      # [R][W][512]
        R, W = rb.shape[0], rb.shape[1]
        out.copy_(rb.view(R, parts, W // parts, SHARE).permute(1, 0, 2, 3))

    def cols(self, block, k, col0, err):
        b = block.numpy()
        W, C = b.shape[0], b.shape[1]
        for j in range(C):
            b[k:, j] = pyref.leopard_encode(b[:k, j])
        leaves = [[pyref.nmt_hash_leaf(_ns(bytes(b[r, j]), r < k and col0 + j < k) + bytes(b[r, j]))
                   for j in range(C)] for r in range(W)]
        for j in range(C):
            if col0 + j < k:
                for r in range(k - 1):
                    if bytes(b[r + 1, j, :NS]) < bytes(b[r, j, :NS]):
                        self._lower(err, (1 << 24) | ((col0 + j) << 12) | (r + 1))
        col_slots = np.zeros((C, SLOT), dtype=np.uint8)
        for j in range(C):
            col_slots[j, :90] = np.frombuffer(pyref.nmt_root_from_nodes([leaves[r][j] for r in range(W)]), np.uint8)
        row_sub = np.zeros((W, SLOT), dtype=np.uint8)
        for r in range(W):
            row_sub[r, :90] = np.frombuffer(pyref.nmt_root_from_nodes(leaves[r]), np.uint8)
        return torch.from_numpy(col_slots), torch.from_numpy(row_sub)

    def combine(self, row_sub_all, parts, k, col_slots_all):
        rs = row_sub_all.numpy()
        W = 2 * k
        rows = [pyref.nmt_root_from_nodes([bytes(rs[g, r, :90]) for g in range(parts)]) for r in range(W)]
        cols = [bytes(col_slots_all.numpy()[j, :90]) for j in range(W)]
        root = pyref.merkle_root(rows + cols)
        return (torch.from_numpy(np.frombuffer(b"".join(rows), np.uint8).reshape(W, 90).copy()),
                torch.from_numpy(np.frombuffer(b"".join(cols), np.uint8).reshape(W, 90).copy()),
                torch.from_numpy(np.frombuffer(root, np.uint8).copy()))
