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
