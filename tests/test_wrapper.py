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
