"""NMT range proofs, RFC-6962 inclusion proofs and GetCommitment -- TEST
INFRASTRUCTURE ONLY (oracle / checker and verifier).

Restates, from their published algorithms (EXT modules, go.mod:9-13):
  * nmt v0.22.0 NamespacedMerkleTree.ProveRange / buildRangeProof: the proof
    nodes are the hashes of the maximal subtrees outside [start, end), in
    depth-first left-to-right order;
  * nmt Proof.VerifyInclusion: recompute the root from the range's leaves and
    the proof nodes;
  * go-square/merkle ProofsFromByteSlices / Proof.Verify (RFC-6962 trails,
    aunts bottom-up);
  * pkg/inclusion/paths.go calculateCommitmentPaths +
    get_commit.go GetCommitment (subtree roots of the ODS half of each row).
Used by tests/test_proofs.py against the GPU proofs.
"""
from __future__ import annotations

import pyref


def split_point(n: int) -> int:
    return pyref._split_point(n)


def nmt_range_proof(leaf_nodes, start: int, end: int):
    """Proof nodes for leaves [start, end) of the NMT over `leaf_nodes`."""
    proof = []

    def root(lo, hi):
        if hi - lo == 1:
            return leaf_nodes[lo]
        k = split_point(hi - lo)
        return pyref.nmt_hash_node(root(lo, lo + k), root(lo + k, hi))

    def rec(lo, hi):
        if hi <= start or lo >= end:
            proof.append(root(lo, hi))
            return
        if hi - lo == 1:
            return
        k = split_point(hi - lo)
        rec(lo, lo + k)
        rec(lo + k, hi)

    rec(0, len(leaf_nodes))
    return proof


def nmt_verify_range(root: bytes, nodes, start: int, end: int, n_leaves: int, range_leaf_nodes) -> bool:
    """Recompute the root of an n_leaves tree from the range's leaf nodes and
    the proof nodes (consumed in order)."""
    it = iter(nodes)
    rl = list(range_leaf_nodes)

    def rec(lo, hi):
        if hi <= start or lo >= end:
            return next(it)
        if hi - lo == 1:
            return rl[lo - start]
        k = split_point(hi - lo)
        return pyref.nmt_hash_node(rec(lo, lo + k), rec(lo + k, hi))

    try:
        got = rec(0, n_leaves)
        leftover = next(it, None)
    except StopIteration:
        return False
    return leftover is None and got == root


def rfc_aunts(items, index: int):
    """merkle.ProofsFromByteSlices(items)[index]: (leaf hash, aunts bottom-up)."""
    def rec(lo, hi):
        if hi - lo == 1:
            return pyref.sha256(b"\x00" + items[lo]), []
        k = split_point(hi - lo)
        if index < lo + k:
            h, a = rec(lo, lo + k)
            return h, a + [pyref.merkle_root(items[lo + k:hi])]
        h, a = rec(lo + k, hi)
        return h, a + [pyref.merkle_root(items[lo:lo + k])]
    return rec(0, len(items))


def rfc_verify(root: bytes, total: int, index: int, leaf_hash: bytes, aunts) -> bool:
    """merkle Proof.Verify / computeHashFromAunts."""
    def compute(idx, tot, leaf, aunts):
        if tot == 1:
            return leaf if not aunts else None
        if not aunts:
            return None
        k = split_point(tot)
        if idx < k:
            left = compute(idx, k, leaf, aunts[:-1])
            return None if left is None else pyref.sha256(b"\x01" + left + aunts[-1])
        right = compute(idx - k, tot - k, leaf, aunts[:-1])
        return None if right is None else pyref.sha256(b"\x01" + aunts[-1] + right)
    return compute(index, total, leaf_hash, list(aunts)) == root


# ------------------------------------------------------------ GetCommitment
def subtree_root_coords(max_depth: int, min_depth: int, start: int, end: int):
    """pkg/inclusion/paths.go calculateSubTreeRootCoordinates (depth, position)."""
    coords = []
    leaf = start
    node = (max_depth, start)
    last_node, last_leaf, rng = node, leaf, 1
    while True:
        if leaf + 1 == end:
            coords.append(node)
            return coords
        if leaf + 1 > end:
            coords.append(last_node)
            leaf = last_leaf + 1
            last_node, last_leaf, node, rng = node, leaf, (max_depth, leaf), 1
        elif not (node[1] % 2 == 0 and node[0] > min_depth):
            coords.append(node)
            leaf += 1
            last_node, last_leaf, node, rng = node, leaf, (max_depth, leaf), 1
        else:
            last_leaf, last_node = leaf, node
            leaf += rng
            rng *= 2
            node = (node[0] - 1, node[1] // 2)


def get_commitment(eds, k: int, start: int, share_len: int, threshold: int = 64) -> bytes:
    """inclusion.GetCommitment from the EDS rows (subtree roots recomputed)."""
    import square
    if start + share_len > k * k:
        raise ValueError("cannot get commitment for blob that doesn't fit in square")
    w = square.subtree_width(share_len, threshold)
    start = -(-start // w) * w
    start_row, end_row = start // k, (start + share_len - 1) // k
    nsi, nei = start % k, start + share_len - end_row * k
    max_depth = k.bit_length() - 1
    min_depth = max_depth - (w.bit_length() - 1)
    roots = []
    for r in range(start_row, end_row + 1):
        s0 = nsi if r == start_row else 0
        e0 = nei if r == end_row else k
        leaves = pyref.erasured_leaves([bytes(c) for c in eds[r]], k, r)
        for depth, pos in subtree_root_coords(max_depth, min_depth, s0, e0):
            size = 1 << (max_depth - depth)
            roots.append(pyref.nmt_root_from_nodes(leaves[pos * size:(pos + 1) * size]))
    return pyref.merkle_root(roots)
