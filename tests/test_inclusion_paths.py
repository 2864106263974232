"""How GetCommitment finds a blob's subtree roots (pkg/inclusion/paths.go
calculateSubTreeRootCoordinates, genSubTreeRootPath,
calculateCommitmentPaths; the cacher's walk, nmt_caching.go:40-78), restated
in oracle/proofs.py and pinned by every known-answer case of the reference's
Test_calculateSubTreeRootCoordinates, Test_genSubTreeRootPath and
Test_calculateCommitPaths (tests/golden/subtree_coords.json,
commit_paths.json, extracted by tests/golden/gen_paths_fixture.py) and by
TestWalkCachedSubTreeRoot's cases.  oracle.get_commitment walks those paths;
the GPU GetCommitment
(cda_square_blob_commitments) is checked against the oracle built on it in
tests/test_proofs.py::test_get_commitment_gpu."""
import json
import os

import pytest

import proofs as opr

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "subtree_coords.json")))["cases"]


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_subtree_root_coordinates(c):
    got = opr.subtree_root_coords(c["max_depth"], c["min_depth"], c["start"], c["end"])
    assert [list(x) for x in got] == c["expected"]


def test_all_cases_extracted():
    assert len(CASES) == 16


# ---- Test_genSubTreeRootPath / Test_calculateCommitPaths (paths_test.go:321-449)
PATHS = json.load(open(os.path.join(HERE, "golden", "commit_paths.json")))


@pytest.mark.parametrize("c", PATHS["gen_path"], ids=lambda c: f"d{c['depth']}p{c['pos']}")
def test_subtree_root_path(c):
    assert opr.subtree_root_path(c["depth"], c["pos"]) == c["expected"]


@pytest.mark.parametrize("c", PATHS["commit_paths"], ids=lambda c: c["name"])
def test_commitment_paths(c):
    paths = opr.commitment_paths(c["square_size"], c["start"], c["blob_len"], PATHS["subtree_root_threshold"])
    for want, i in zip(c["expected_paths"], c["expected_indexes"]):
        assert paths[i] == (want["row"], want["walk"])
    # the reference test's uniqueness check (pathToString)
    keys = [str(r) + "".join("r" if s else "l" for s in w) for r, w in paths]
    assert len(set(keys)) == len(keys)


def test_all_path_cases_extracted():
    assert len(PATHS["gen_path"]) == 6 and len(PATHS["commit_paths"]) == 8


# ---- TestWalkCachedSubTreeRoot (nmt_caching_test.go:19-115) on the oracle's walk
def test_walk_cached_subtree_root():
    import pyref
    # appns.MustNewV0(1 x 10).Bytes() (version 0, 18 zero bytes, the 10-byte ID) || "data"
    data = b"\x00" + b"\x00" * 18 + b"\x01" * 10 + b"data"

    def leaves(n):
        return pyref.erasured_leaves([data] * n, 8, 0)

    short_root = pyref.nmt_root_from_nodes(leaves(2))
    tall_root = pyref.nmt_root_from_nodes(leaves(4))
    tree = leaves(8)
    L, R = opr.WALK_LEFT, opr.WALK_RIGHT
    for walk, want in [([L, L], short_root), ([L, R], short_root), ([R, L], short_root), ([R, R], short_root),
                       ([L], tall_root), ([R], tall_root)]:
        assert opr.walk_subtree_root(tree, walk) == want
    with pytest.raises(KeyError, match="did not find sub tree root"):
        opr.walk_subtree_root(tree, [R, R, R, R])


# ---- TestEDSSubRootCacher (nmt_caching_test.go:117-137) on the resident square
@pytest.mark.gpu
@pytest.mark.parametrize("k", [8, 32])
def test_eds_subtree_root_cacher(ctx, k):
    """getSubTreeRoot(dah, row, [L, L, L]) of every ODS row equals the root of
    an erasured tree over the row's first 2k >> 3 shares (the reference's
    calculateSubTreeRoots), and every walk equals the oracle's walk on the
    row's leaves; the cache's errors."""
    import numpy as np
    import pyref
    from celestia_da import CdaError, testfactory
    from celestia_da import proof as gpr
    ods = testfactory.random_square(k, 9)
    eds = pyref.extend_square(ods.reshape(k, k, 512))
    sq = gpr.ResidentSquare(ods)
    try:
        L, R = opr.WALK_LEFT, opr.WALK_RIGHT
        n = 2 * k >> 3
        for i in range(k):
            want = pyref.axis_root([bytes(c) for c in eds[i, :n]], n, 0)   # calculateSubTreeRoots
            assert sq.subtree_root(i, [L, L, L]) == want
        rng = np.random.default_rng(1)
        depth = (2 * k).bit_length() - 1
        for _ in range(24):
            r = int(rng.integers(2 * k))
            walk = [bool(b) for b in rng.integers(0, 2, int(rng.integers(0, depth + 1)))]
            leaves = pyref.erasured_leaves([bytes(c) for c in eds[r]], k, r)
            assert sq.subtree_root(r, walk) == opr.walk_subtree_root(leaves, walk)
        assert sq.subtree_root(0, []) == sq.dah()[0][0]
        with pytest.raises(CdaError, match="did not find sub tree root"):
            sq.subtree_root(0, [L] * (depth + 1))
        with pytest.raises(CdaError, match=f"row exceeds range of cache: max {2 * k} got {2 * k}"):
            sq.subtree_root(2 * k, [L])
    finally:
        sq.close()
