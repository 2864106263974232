"""calculateSubTreeRootCoordinates (pkg/inclusion/paths.go), the coordinate
walk GetCommitment's subtree roots follow, restated in oracle/proofs.py
(subtree_root_coords) and pinned by every known-answer case of the
reference's Test_calculateSubTreeRootCoordinates
(tests/golden/subtree_coords.json, extracted by
tests/golden/gen_paths_fixture.py).  The GPU GetCommitment
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
