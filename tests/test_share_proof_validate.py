"""ShareProof.Validate / RowProof.Validate (pkg/proof/share_proof.go:16-78,
row_proof.go:13-51) restated in the oracle (oracle/proofs.py
share_proof_validate) and pinned by the reference's own vector: the valid
one-share proof and data root of pkg/proof/share_proof_test.go:77-93 and
row_proof_test.go:68-89 (tests/golden/share_proof_valid.json, extracted by
tests/golden/gen_share_proof_fixture.py).  The cases are the reference
tests' (TestShareProofValidate, TestRowProofValidate).  The GPU proofs are
validated with the same function in test_proofs.py / test_tx_proofs.py.
"""
import copy
import json
import os

import proofs as opr

HERE = os.path.dirname(os.path.abspath(__file__))


def fixture():
    d = json.load(open(os.path.join(HERE, "golden", "share_proof_valid.json")))
    h = bytes.fromhex
    sp = {"data": [h(x) for x in d["data"]],
          "share_proofs": [{"start": p["start"], "end": p["end"], "nodes": [h(n) for n in p["nodes"]]}
                           for p in d["share_proofs"]],
          "namespace_id": h(d["namespace_id"]), "namespace_version": d["namespace_version"],
          "row_proof": {"row_roots": [h(r) for r in d["row_proof"]["row_roots"]],
                        "proofs": [{"total": p["total"], "index": p["index"], "leaf_hash": h(p["leaf_hash"]),
                                    "aunts": [h(a) for a in p["aunts"]]} for p in d["row_proof"]["proofs"]],
                        "start_row": d["row_proof"]["start_row"], "end_row": d["row_proof"]["end_row"]}}
    return sp, h(d["root"])


def to_dict(p):
    """celestia_da.proof.ShareProof -> the oracle's dict form."""
    return {"data": list(p.data),
            "share_proofs": [{"start": s.start, "end": s.end, "nodes": list(s.nodes)} for s in p.share_proofs],
            "namespace_id": p.namespace_id, "namespace_version": p.namespace_version,
            "row_proof": {"row_roots": list(p.row_proof.row_roots),
                          "proofs": [{"total": q.total, "index": q.index, "leaf_hash": q.leaf_hash, "aunts": q.aunts}
                                     for q in p.row_proof.proofs],
                          "start_row": p.row_proof.start_row, "end_row": p.row_proof.end_row}}


def test_share_proof_validate_cases():
    sp, root = fixture()
    assert opr.share_proof_validate(sp, root) is None
    assert opr.share_proof_validate({"data": None}, root) == "empty share proof"
    bad = copy.deepcopy(sp)
    bad["share_proofs"] = bad["share_proofs"] * 2            # mismatchedShareProofs
    assert opr.share_proof_validate(bad, root).startswith("the number of share proofs 2 must equal")
    bad = copy.deepcopy(sp)
    bad["data"] = bad["data"] * 2                            # mismatchedShares
    assert opr.share_proof_validate(bad, root) == \
        "the number of shares 2 must equal the number of shares in share proofs 1"
    assert opr.share_proof_validate(sp, bytes(32)) == "row proof failed to verify"   # incorrectRoot


def test_row_proof_validate_cases():
    sp, root = fixture()
    rp = sp["row_proof"]
    assert opr.row_proof_validate(rp, root) is None
    assert opr.row_proof_validate(rp, bytes(32)) == "row proof failed to verify"
    for field, value, want in [
        ("row_roots", [], "the number of rows 1 must equal the number of row roots 0"),     # mismatchedRowRoots
        ("proofs", [], "the number of proofs 0 must equal the number of row roots 1"),      # mismatchedProofs
        ("end_row", 10, "the number of rows 11 must equal the number of row roots 1"),      # mismatchedRows
    ]:
        bad = copy.deepcopy(rp)
        bad[field] = value
        assert opr.row_proof_validate(bad, root) == want, field


def test_tampering_is_caught():
    sp, root = fixture()
    for path in ("data", "nodes", "leaf_hash", "aunts", "row_roots"):
        bad = copy.deepcopy(sp)
        if path == "data":
            d = bytearray(bad["data"][0]); d[100] ^= 1; bad["data"][0] = bytes(d)
        elif path == "nodes":
            n = bytearray(bad["share_proofs"][0]["nodes"][2]); n[-1] ^= 1; bad["share_proofs"][0]["nodes"][2] = bytes(n)
        elif path == "leaf_hash":
            lh = bytearray(bad["row_proof"]["proofs"][0]["leaf_hash"]); lh[0] ^= 1
            bad["row_proof"]["proofs"][0]["leaf_hash"] = bytes(lh)
        elif path == "aunts":
            a = bytearray(bad["row_proof"]["proofs"][0]["aunts"][3]); a[5] ^= 1
            bad["row_proof"]["proofs"][0]["aunts"][3] = bytes(a)
        else:
            r = bytearray(bad["row_proof"]["row_roots"][0]); r[-1] ^= 1; bad["row_proof"]["row_roots"][0] = bytes(r)
        assert opr.share_proof_validate(bad, root) is not None, path


def test_generic_nmt_matches_29_byte_rules():
    """The generic-namespace hashing equals pyref's 29-byte NMT rules."""
    import pyref
    a, b = pyref.nmt_hash_leaf(b"\x00" * 28 + b"\x01" + b"x" * 512), pyref.nmt_hash_leaf(b"\xff" * 29 + b"y" * 512)
    assert opr._nmt_node(29, a, b) == pyref.nmt_hash_node(a, b)
    assert opr._nmt_leaf(29, b"\x00" * 28 + b"\x07" + b"z" * 512) == pyref.nmt_hash_leaf(b"\x00" * 28 + b"\x07" + b"z" * 512)
