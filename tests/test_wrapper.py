"""pkg/wrapper conventions (ErasuredNamespacedMerkleTree, NewConstructor).

Mirrors /root/reference/pkg/wrapper/nmt_wrapper_test.go:
  * TestPushErasuredNamespacedMerkleTree (:19-42): 2k erasured shares push
    cleanly at k = 8 and 128;
  * TestErasureNamespacedMerkleTreePushErrors (:91-128): push past the square,
    out of namespace order, too short for a namespace -> error;
  * TestErasuredNamespacedMerkleTreeEmptyRoot (:76-89): empty roots are equal
    whatever the parameters (NmtHasher.EmptyRoot);
  * TestRootErasuredNamespacedMerkleTree (:49-73): the erasured root differs
    from a plain NMT root of the same data (checked on the oracle; the GPU
    erasured roots are pinned to the oracle by test_gpu_parity.py);
  * TestComputeExtendedDataSquare (:130-137) on the GPU.
The push rules are host logic (celestia_da/wrapper.py); the erasure data is
generated with the oracle encoder (test infrastructure only).
"""
import numpy as np
import pytest

import pyref
from celestia_da import wrapper


def erasured_data(k, seed=1):
    """generateErasuredData (:139-152): k random namespaced shares, sorted,
    then their Leopard parity -> 2k shares."""
    shares = np.stack([pyref.random_namespaced_square(1, seed * 1000 + i)[0] for i in range(k)])
    shares = shares[np.lexsort(shares.T[::-1])]
    parity = pyref.leopard_encode(shares)
    return [bytes(s) for s in shares] + [bytes(p) for p in parity]


@pytest.mark.parametrize("k", [8, 128])
def test_push_erasured_shares(k):
    tree = wrapper.new_erasured_namespaced_merkle_tree(k, 0)
    for d in erasured_data(k):
        tree.push(d)
    assert tree.share_index == 2 * k


def test_push_errors():
    k = 16
    full = erasured_data(k)
    over = full + full[-1:]               # generateErasuredData(k+1): more than 2k pushes
    rev = sorted(erasured_data(k), reverse=True)
    for data, msg in ((over, "pushed past predetermined square size"),
                      (rev, "lexicographically ordered"),
                      ([b"\x01"], "too short to contain namespace")):
        tree = wrapper.new_erasured_namespaced_merkle_tree(k, 0)
        err = None
        for d in data:
            try:
                tree.push(d)
            except ValueError as e:
                err = e
                break
        assert err is not None and msg in str(err), (msg, err)


def test_constructor_rejects_zero_square():
    with pytest.raises(ValueError):
        wrapper.new_erasured_namespaced_merkle_tree(0, 0)


def test_empty_roots_equal():
    r1 = wrapper.new_erasured_namespaced_merkle_tree(1, 0).root()
    r2 = wrapper.new_erasured_namespaced_merkle_tree(2, 1).root()
    assert r1 == r2 == wrapper.EMPTY_ROOT == pyref.nmt_empty_root()


def test_erasured_root_differs_from_plain_nmt():
    k = 8
    data = erasured_data(k)[:k]
    erasured = pyref.nmt_root_from_nodes(pyref.erasured_leaves(data, k, 0))
    plain = pyref.nmt_root_from_nodes([pyref.nmt_hash_leaf(d) for d in data])
    assert erasured != plain
    # a parity-half push uses ParitySharesNamespace
    full = erasured_data(k)
    leaves = pyref.erasured_leaves(full, k, 0)
    assert leaves[k][:29] == wrapper.PARITY_SHARES_NAMESPACE and leaves[k - 1][:29] == full[k - 1][:29]


@pytest.mark.gpu
def test_compute_extended_data_square(ctx):
    from celestia_da import rsmt2d
    k = 4
    ods = pyref.random_namespaced_square(k, 3)
    eds = rsmt2d.compute_extended_data_square(ods, rsmt2d.LeoRSCodec(ctx), wrapper.new_constructor(k))
    rows = eds.row_roots()
    assert len(rows) == 2 * k
    assert rows[0] == pyref.axis_root(eds.row(0), k, 0)


# ---- standalone trees on the GPU (cda_nmt_axis_root / cda_nmt_prove_range) ----
import proofs  # noqa: E402  (oracle: nmt ProveRange / VerifyInclusion restatement)
from celestia_da import testfactory  # noqa: E402


def gpu_erasured_data(ctx, k, seed=1):
    """generateErasuredData (:139-152) with the GPU codec: k random namespaced
    shares (GenerateRandNamespacedRawData, sorted) + LeoRSCodec.Encode."""
    from celestia_da import rsmt2d
    raw = testfactory.random_namespaced_shares(k, 500 + seed)
    parity = rsmt2d.LeoRSCodec(ctx).encode(raw)
    assert np.array_equal(parity, pyref.leopard_encode(raw)), "codec parity differs from the oracle"
    return [bytes(s) for s in raw] + [bytes(p) for p in parity]


@pytest.mark.gpu
def test_root_erasured_tree_on_gpu(ctx):
    """TestRootErasuredNamespacedMerkleTree (:49-73): 8 pushes into a k=8 tree;
    the GPU root equals the oracle's erasured root and differs from a plain
    NMT root of the same data."""
    size = 8
    data = [bytes(s) for s in testfactory.random_namespaced_shares(size, 77)]
    tree = wrapper.new_erasured_namespaced_merkle_tree(size, 0, ctx)
    for d in data:
        tree.push(d)
    root = tree.root()
    assert root == pyref.nmt_root_from_nodes(pyref.erasured_leaves(data, size, 0))
    assert root != pyref.nmt_root_from_nodes([pyref.nmt_hash_leaf(d) for d in data])   # nmtStandard.Push(d)


@pytest.mark.gpu
@pytest.mark.parametrize("k", range(1, 17))
def test_prove_range_on_gpu(ctx, k):
    """TestErasuredNamespacedMerkleTree_ProveRange (:152-180), squareSize 1..16
    (non-powers of two included: nmt's RFC-6962 split, Leopard's padded
    encode): every single-leaf proof equals the oracle's nodes and verifies
    against the root with the leaf's namespace (parity namespace in the
    parity half)."""
    data = gpu_erasured_data(ctx, k, seed=k)
    tree = wrapper.new_erasured_namespaced_merkle_tree(k, 0, ctx)
    for d in data:
        tree.push(d)
    leaves = pyref.erasured_leaves(data, k, 0)
    root = tree.root()
    assert root == pyref.nmt_root_from_nodes(leaves)
    for i in range(len(data)):
        nodes = tree.prove_range(i, i + 1)
        assert nodes, "proof must not be empty"
        assert nodes == proofs.nmt_range_proof(leaves, i, i + 1)
        ns = data[i][:29] if i < k else wrapper.PARITY_SHARES_NAMESPACE
        assert proofs.nmt_verify_range(root, nodes, i, i + 1, len(data), [pyref.nmt_hash_leaf(ns + data[i])])
    with pytest.raises(Exception, match="invalid proof range"):
        tree.prove_range(3, 3)


@pytest.mark.gpu
@pytest.mark.parametrize("k,n_cells,cell_len,axes", [
    (8, 16, 512, [0, 1, 2, 3]),          # rows of a square: fast path
    (8, 16, 512, [9, 3, 12]),            # scattered axes: generic kernels
    (8, 11, 512, [0, 8]),                # ragged leaf count
    (4, 8, 64, [1, 2]),                  # 64-B chunks (rsmt2d chunk size)
    (128, 256, 512, list(range(64, 192))),   # pkg/inclusion/nmt_caching.go: many rows at once
])
def test_axis_roots_batch_on_gpu(ctx, k, n_cells, cell_len, axes):
    rng = np.random.default_rng(k * 1000 + n_cells)
    cells = rng.integers(0, 256, (len(axes), n_cells, cell_len), dtype=np.uint8)
    cells[:, :, :29] = 0
    cells[:, :, 28] = np.arange(n_cells, dtype=np.uint8)[None, :]   # ordered namespaces
    roots = wrapper.axis_roots(cells, k, axes, ctx)
    for t, ax in enumerate(axes):
        assert roots[t].tobytes() == pyref.axis_root(list(cells[t]), k, ax), (t, ax)


@pytest.mark.gpu
def test_axis_roots_push_order_on_gpu(ctx):
    from celestia_da import PushOrderError
    k = 8
    cells = np.zeros((2, 16, 512), dtype=np.uint8)
    cells[:, :, 28] = np.arange(16, dtype=np.uint8)[None, :]
    cells[1, 5, 28], cells[1, 6, 28] = 6, 5
    with pytest.raises(PushOrderError, match="lexicographically ordered"):
        wrapper.axis_roots(cells, k, [0, 1], ctx)
    axis, idx, pos = ctx.push_order_detail()
    assert (idx, pos) == (1, 6)


@pytest.mark.gpu
def test_seeded_tree_recomputes_when_fed_other_cells(ctx):
    """A tree seeded with the square's GPU root returns it only for the cells
    it was seeded for; pushing changed cells gives the root of what was
    pushed (not a stale seed)."""
    from celestia_da import da
    k = 4
    ods = testfactory.random_square(k, 3)
    eds = da.extend_shares(ods)
    seeded_root = eds.row_roots()[1]
    row = eds.row(1)
    same = wrapper.new_erasured_namespaced_merkle_tree(k, 1, ctx)
    same.seed(seeded_root, [np.frombuffer(c, dtype=np.uint8) for c in row])
    for c in row:
        same.push(c)
    assert same.root() == seeded_root
    changed = list(row)
    changed[k + 1] = bytes(512)            # a parity cell altered after extension
    t = wrapper.new_erasured_namespaced_merkle_tree(k, 1, ctx)
    t.seed(seeded_root, [np.frombuffer(c, dtype=np.uint8) for c in row])
    for c in changed:
        t.push(c)
    assert t.root() == pyref.axis_root(changed, k, 1) != seeded_root


@pytest.mark.gpu
def test_cell_rewritten_in_place_after_extend_shares_gets_recomputed_root(ctx):
    """a cell rewritten IN PLACE (same backing array) after
    ExtendShares must not return the extension's stale GPU root -- rsmt2d
    hashes the cells when RowRoots/ColRoots is first called
    (pkg/da/data_availability_header.go:44-63 -> computeRoots), so the DAH is
    that of the rewritten square, and a tree seeded before the rewrite drops
    its seed."""
    from celestia_da import da
    k = 8
    W = 2 * k
    ods = testfactory.random_square(k, 21)
    eds = da.extend_shares(ods)
    arr = eds.array()
    seeded_row = eds.row(W - 1)
    arr[W - 1, W - 2, 100:140] ^= 0x5A            # parity cell of row W-1 / column W-2, in place
    rows, cols, _ = pyref.dah_from_eds(np.asarray(arr).reshape(W, W, 512).copy())
    dah = da.new_data_availability_header(eds)
    assert dah.row_roots == [bytes(r) for r in rows] and dah.column_roots == [bytes(c) for c in cols]
    assert dah.row_roots[W - 1] == pyref.axis_root([bytes(c) for c in arr[W - 1]], k, W - 1)
    # a standalone tree seeded with the row as it was, then fed the same
    # (now rewritten) buffer views, recomputes
    t = wrapper.new_erasured_namespaced_merkle_tree(k, W - 1, ctx)
    t.seed(b"\x00" * 90, [np.frombuffer(c, dtype=np.uint8) for c in seeded_row])
    for c in range(W):
        t.push(arr[W - 1, c])
    assert t.root() == dah.row_roots[W - 1]


@pytest.mark.gpu
def test_axis_roots_reports_every_violating_tree(ctx):
    """cda_nmt_axis_roots' per-tree status must flag EVERY tree
    that breaks push order, not only the first one (nmt Push
    ErrInvalidPushOrder per tree; pkg/wrapper/nmt_wrapper.go:93-114)."""
    k = 8
    ods = testfactory.random_square(k, 4).reshape(k, k, 512)
    rows = np.ascontiguousarray(ods[:, :, :].copy())
    parity = np.zeros((k, k, 512), dtype=np.uint8)
    cells = np.concatenate([rows, parity], axis=1)          # k trees (rows 0..k-1) of 2k cells
    bad = (1, 4, 6)
    for t in bad:                                          # swap two Q0 cells: namespace out of order
        cells[t, [2, 5]] = cells[t, [5, 2]]
    n_trees, n_cells, _ = cells.shape
    out = np.empty((n_trees, 90), dtype=np.uint8)
    status = np.empty(n_trees, dtype=np.int32)
    import ctypes as C
    from celestia_da._lib import CDA_ERR_PUSH_ORDER, ptr
    axes = np.arange(n_trees, dtype=np.uint32)
    rc = ctx.lib.cda_nmt_axis_roots(ctx.h, ptr(np.ascontiguousarray(cells)), 512, n_cells, n_trees, k,
                                    axes.ctypes.data_as(C.POINTER(C.c_uint32)), ptr(out),
                                    status.ctypes.data_as(C.POINTER(C.c_int32)))
    assert rc == CDA_ERR_PUSH_ORDER
    want = [CDA_ERR_PUSH_ORDER if t in bad else 0 for t in range(n_trees)]
    assert status.tolist() == want
    for t in range(n_trees):
        if t not in bad:
            assert out[t].tobytes() == pyref.axis_root([bytes(c) for c in cells[t]], k, t)
