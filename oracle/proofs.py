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
  * pkg/proof/share_proof.go:16-78 ShareProof.Validate / VerifyProof and
    row_proof.go:13-51 RowProof.Validate, over nmt's VerifyInclusion with the
    namespace size taken from the proof (the reference's fixture uses 33-byte
    namespaces), pinned by that fixture (tests/golden/share_proof_valid.json).
Used by tests/test_proofs.py and tests/test_tx_proofs.py against the GPU proofs.
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


# ------------------------------------------------- ShareProof.Validate (generic ns)
def _nmt_leaf(nsz: int, ndata: bytes) -> bytes:
    ns = ndata[:nsz]
    return ns + ns + pyref.sha256(b"\x00" + ndata)


def _nmt_node(nsz: int, left: bytes, right: bytes) -> bytes:
    lmin, lmax = left[:nsz], left[nsz:2 * nsz]
    rmin, rmax = right[:nsz], right[nsz:2 * nsz]
    mx = lmax if rmin == b"\xff" * nsz else rmax      # IgnoreMaxNamespace(true)
    return lmin + mx + pyref.sha256(b"\x01" + left + right)


def _nmt_split(n: int) -> int:
    """nmt getSplitPoint: the largest power of two below n (0 for n = 1)."""
    k = 1 << (n.bit_length() - 1)
    return k >> 1 if k == n else k


def nmt_verify_inclusion(root: bytes, nodes, start: int, end: int, nid: bytes, leaves) -> bool:
    """nmt Proof.VerifyInclusion (ignore-max-namespace proofs): leaf hashes of
    nid || leaf, the subtree that holds the range (size 2 * getSplitPoint(end))
    from them and the proof nodes met on the way, then the remaining nodes
    folded in on the right."""
    nsz = len(nid)
    hashes = [_nmt_leaf(nsz, nid + bytes(x)) for x in leaves]
    rest = list(nodes)

    def pop(a):
        return a.pop(0) if a else None

    def compute(lo, hi):
        if hi - lo == 1:
            return pop(hashes) if start <= lo < end else pop(rest)
        if hi <= start or lo >= end:
            return pop(rest)
        k = _nmt_split(hi - lo)
        left, right = compute(lo, lo + k), compute(lo + k, hi)
        return left if right is None else _nmt_node(nsz, left, right)

    h = compute(0, max(1, 2 * _nmt_split(end)))
    while rest:
        h = _nmt_node(nsz, h, rest.pop(0))
    return h == root


def merkle_proof_verify(root: bytes, total: int, index: int, leaf_hash: bytes, aunts, leaf: bytes) -> bool:
    """go-square/merkle Proof.Verify: the leaf hash must be the leaf's, then the trail."""
    if total < 0 or index < 0 or pyref.sha256(b"\x00" + leaf) != leaf_hash:
        return False
    return rfc_verify(root, total, index, leaf_hash, aunts)


def row_proof_validate(rp: dict, root: bytes):
    """RowProof.Validate(root) (row_proof.go:13-27): None or the error text."""
    rows = rp["end_row"] - rp["start_row"] + 1
    if rows != len(rp["row_roots"]):
        return f"the number of rows {rows} must equal the number of row roots {len(rp['row_roots'])}"
    if len(rp["proofs"]) != len(rp["row_roots"]):
        return f"the number of proofs {len(rp['proofs'])} must equal the number of row roots {len(rp['row_roots'])}"
    for p, r in zip(rp["proofs"], rp["row_roots"]):
        if not merkle_proof_verify(root, p["total"], p["index"], p["leaf_hash"], p["aunts"], r):
            return "row proof failed to verify"
    return None


def share_proof_validate(sp: dict, root: bytes):
    """ShareProof.Validate(root): None when valid, else the reference's error
    text.  sp: {data, share_proofs [{start, end, nodes}], namespace_id,
    namespace_version, row_proof {row_roots, proofs [{total, index,
    leaf_hash, aunts}], start_row, end_row}} with bytes values."""
    if not sp.get("data"):
        return "empty share proof"
    n_in_proofs = sum(p["end"] - p["start"] for p in sp["share_proofs"])
    rp = sp["row_proof"]
    if len(sp["share_proofs"]) != len(rp["row_roots"]):
        return (f"the number of share proofs {len(sp['share_proofs'])} must equal the number of row roots "
                f"{len(rp['row_roots'])}")
    if len(sp["data"]) != n_in_proofs:
        return f"the number of shares {len(sp['data'])} must equal the number of shares in share proofs {n_in_proofs}"
    for p in sp["share_proofs"]:
        if p["start"] < 0:
            return "proof index cannot be negative"
        if p["end"] - p["start"] <= 0:
            return "proof total must be positive"
    err = row_proof_validate(rp, root)
    if err is not None:
        return err
    # VerifyProof
    if sp["namespace_version"] > 255:
        return "share proof failed to verify"
    nid = bytes([sp["namespace_version"]]) + sp["namespace_id"]
    cursor = 0
    for p, r in zip(sp["share_proofs"], rp["row_roots"]):
        used = p["end"] - p["start"]
        if not nmt_verify_inclusion(r, p["nodes"], p["start"], p["end"], nid, sp["data"][cursor:cursor + used]):
            return "share proof failed to verify"
        cursor += used
    return None


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


WALK_LEFT, WALK_RIGHT = False, True      # pkg/inclusion/nmt_caching.go WalkInstruction


def subtree_root_path(depth: int, pos: int):
    """pkg/inclusion/paths.go genSubTreeRootPath: the walk from a tree's root
    to node (depth, pos), most significant position bit first."""
    return [bool(pos & (1 << i)) for i in range(depth - 1, -1, -1)]


def commitment_paths(k: int, start: int, share_len: int, threshold: int = 64):
    """pkg/inclusion/paths.go calculateCommitmentPaths: (row, walk) of every
    subtree root a blob's commitment uses, walks relative to the ODS half of
    the row tree."""
    import square
    start = square.next_share_index(start, share_len, threshold)
    start_row, end_row = start // k, (start + share_len - 1) // k
    nsi, nei = start % k, start + share_len - end_row * k
    max_depth = k.bit_length() - 1
    min_depth = max_depth - (square.subtree_width(share_len, threshold).bit_length() - 1)
    paths = []
    for r in range(start_row, end_row + 1):
        s0 = nsi if r == start_row else 0
        e0 = nei if r == end_row else k
        for depth, pos in subtree_root_coords(max_depth, min_depth, s0, e0):
            paths.append((r, subtree_root_path(depth, pos)))
    return paths


def walk_subtree_root(leaf_nodes, walk):
    """EDSSubTreeRootCacher.walk (pkg/inclusion/nmt_caching.go:40-78) on a
    row tree given by its leaf nodes: the node reached from the root by the
    walk; a walk deeper than the tree fails like the cache miss does."""
    lo, hi = 0, len(leaf_nodes)
    for step in walk:
        if hi - lo < 2:
            raise KeyError("did not find sub tree root")
        mid = lo + split_point(hi - lo)
        lo, hi = (mid, hi) if step else (lo, mid)
    return pyref.nmt_root_from_nodes(leaf_nodes[lo:hi])


def get_commitment(eds, k: int, start: int, share_len: int, threshold: int = 64) -> bytes:
    """inclusion.GetCommitment (pkg/inclusion/get_commit.go:12-30) from the EDS
    rows: each path is prefixed with WalkLeft (the ODS half of the 2k-leaf row
    tree) and walked down that row's tree."""
    if start + share_len > k * k:
        raise ValueError("cannot get commitment for blob that doesn't fit in square")
    roots = []
    for r, walk in commitment_paths(k, start, share_len, threshold):
        leaves = pyref.erasured_leaves([bytes(c) for c in eds[r]], k, r)
        roots.append(walk_subtree_root(leaves, [WALK_LEFT] + walk))
    return pyref.merkle_root(roots)
