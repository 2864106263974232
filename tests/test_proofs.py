"""NMT share-inclusion proofs and GetCommitment from resident squares
(SURVEY.md 8(f) row 3).

Checks:
  * CPU: the oracle's proof restatements are self-consistent (a range proof
    verifies against the row root, RFC-6962 aunts verify against the data
    root) and its GetCommitment (pkg/inclusion/paths.go restated) equals
    CreateCommitment for every blob of constructed squares, which is the
    reference's own invariant (ProcessProposal accepts only squares whose blob
    layout reproduces the PFB commitments);
  * GPU: cda_square_share_proof returns exactly the oracle's nodes, aunts and
    shares, and they verify against the square's roots; cda_square_blob_
    commitments equals the PFB commitments.
"""
import numpy as np
import pytest

import coracle
import inclusion as oinc
import proofs as opr
import pyref
import square as osq
from celestia_da import CdaError, blobfactory
from celestia_da import proof as gpr
from test_share_proof_validate import to_dict


def constructed_square(seed, max_ss=32, n_blob_txs=12, blob_size=(1, 6000)):
    txs = blobfactory.random_block(seed, 3, n_blob_txs, (1, 2), blob_size, 2)
    shares, ss, kept, idx = osq.builder(txs, max_ss, 64, "build")
    ods = np.frombuffer(b"".join(shares), dtype=np.uint8).reshape(-1, 512).copy()
    blobs = []   # (start share, share count, namespace, data) in PFB order
    j = 0
    for t in kept:
        bt = osq.unmarshal_blob_tx(txs[t])
        if bt is None:
            continue
        for b in bt[1]:
            ns = bytes([b["namespace_version"]]) + b["namespace_id"]
            blobs.append((idx[j], osq.sparse_share_count(len(b["data"])), ns, b["data"]))
            j += 1
    return ods, ss, blobs


def oracle_eds(ods, k):
    eds, rows, cols, root = coracle.extend_dah(ods)
    return eds.reshape(2 * k, 2 * k, 512), [bytes(r) for r in rows], [bytes(c) for c in cols], root


def ranges(k, blobs):
    out = [(0, 1), (k - 1, k + 1), (3, 2 * k + 5), (k * k - 1, k * k), (0, k * k)]
    out += [(s, s + n) for s, n, _, _ in blobs[:6]]
    return out


# ------------------------------------------------------------------ CPU tests
def test_oracle_proofs_self_consistent():
    ods, k, blobs = constructed_square(1, 16, 6, (1, 3000))
    eds, rows, cols, root = oracle_eds(ods, k)
    items = rows + cols
    for s, e in [(0, 1), (3, 9), (0, k), (k - 1, k)]:
        leaves = pyref.erasured_leaves([bytes(c) for c in eds[0]], k, 0)
        nodes = opr.nmt_range_proof(leaves, s, e)
        assert opr.nmt_verify_range(rows[0], nodes, s, e, 2 * k, leaves[s:e])
        assert not opr.nmt_verify_range(rows[1], nodes, s, e, 2 * k, leaves[s:e])
    for i in (0, 1, k, 4 * k - 1):
        lh, aunts = opr.rfc_aunts(items, i)
        assert opr.rfc_verify(root, 4 * k, i, lh, aunts)
        assert not opr.rfc_verify(root, 4 * k, i ^ 1, lh, aunts)


def test_oracle_get_commitment_equals_create_commitment():
    ods, k, blobs = constructed_square(2, 32, 10, (1, 9000))
    eds, _, _, _ = oracle_eds(ods, k)
    assert blobs
    for start, n, ns, data in blobs:
        assert opr.get_commitment(eds, k, start, n) == oinc.create_commitment(ns, data)


# ------------------------------------------------------------------ GPU tests
@pytest.mark.gpu
@pytest.mark.parametrize("seed,max_ss", [(3, 16), (4, 32), (5, 64)])
def test_share_proofs_gpu(ctx, seed, max_ss):
    ods, k, blobs = constructed_square(seed, max_ss, 8 * max_ss // 16, (1, 6000 * max_ss // 16))
    eds, rows, cols, root = oracle_eds(ods, k)
    sq = gpr.ResidentSquare(ods)
    try:
        g_rows, g_cols, g_root = sq.dah()
        assert (g_rows, g_cols, g_root) == (rows, cols, root)
        assert np.array_equal(sq.eds(), eds)
        items = rows + cols
        for s, e in ranges(k, blobs):
            p = sq.share_proof(bytes(eds[s // k][s % k][:29]), s, e)
            if len({bytes(eds[i // k][i % k][:29]) for i in range(s, e)}) == 1:   # one namespace: Validate applies
                assert opr.share_proof_validate(to_dict(p), root) is None
            r0, r1 = s // k, (e - 1) // k
            assert (p.row_proof.start_row, p.row_proof.end_row) == (r0, r1)
            assert b"".join(p.data) == eds.reshape(-1, 512)[0:0].tobytes() + b"".join(
                bytes(eds[i // k][i % k]) for i in range(s, e))
            for i, r in enumerate(range(r0, r1 + 1)):
                sp = p.share_proofs[i]
                leaves = pyref.erasured_leaves([bytes(c) for c in eds[r]], k, r)
                assert sp.nodes == opr.nmt_range_proof(leaves, sp.start, sp.end)
                assert opr.nmt_verify_range(rows[r], sp.nodes, sp.start, sp.end, 2 * k, leaves[sp.start:sp.end])
                rp = p.row_proof.proofs[i]
                lh, aunts = opr.rfc_aunts(items, r)
                assert (rp.total, rp.index, rp.leaf_hash, rp.aunts) == (4 * k, r, lh, aunts)
                assert opr.rfc_verify(root, rp.total, rp.index, rp.leaf_hash, rp.aunts)
                assert p.row_proof.row_roots[i] == rows[r]
        with pytest.raises(CdaError):
            sq.share_proof(b"\x00" * 29, 0, k * k + 1)
    finally:
        sq.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,max_ss", [(6, 32), (7, 64), (8, 128)])
def test_get_commitment_gpu(ctx, seed, max_ss):
    ods, k, blobs = constructed_square(seed, max_ss, 6 * max_ss // 16, (1, 8000 * max_ss // 16))
    sq = gpr.ResidentSquare(ods)
    try:
        got = sq.blob_commitments([b[0] for b in blobs], [b[1] for b in blobs])
        for (start, n, ns, data), c in zip(blobs, got):
            assert c == oinc.create_commitment(ns, data)
        with pytest.raises(CdaError, match="doesn't fit"):
            sq.blob_commitments([k * k - 1], [2])
    finally:
        sq.close()


@pytest.mark.gpu
def test_resident_square_k1(ctx):
    """The smallest square (MinDataAvailabilityHeader's tail-padding share,
    data_availability_header_test.go:27-32) through every resident-square
    entry point: the golden data root, the one-share proof, the walks of a
    two-leaf row tree, a one-share commitment."""
    from celestia_da import da
    from test_share_proof_validate import to_dict
    share = da.tail_padding_share()
    sq = gpr.ResidentSquare(np.frombuffer(share, dtype=np.uint8).copy())
    try:
        rows, cols, root = sq.dah()
        assert root.hex() == "3d96b7d238e7e0456f6af8e7cdf0a67bd6cf9c2089ecb559c659dcaa1f880353"
        p = sq.share_proof(share[:29], 0, 1)
        assert opr.share_proof_validate(to_dict(p), root) is None and p.data == [share]
        leaves = pyref.erasured_leaves([share, bytes(sq.eds()[0][1])], 1, 0)
        assert sq.subtree_root(0, []) == rows[0]
        assert sq.subtree_root(0, [False]) == leaves[0] and sq.subtree_root(1, [True]) == pyref.erasured_leaves(
            [bytes(c) for c in sq.eds()[1]], 1, 1)[1]
        assert sq.blob_commitments([0], [1]) == [opr.get_commitment(sq.eds(), 1, 0, 1)]
    finally:
        sq.close()


@pytest.mark.gpu
def test_resident_square_k512():
    """The largest square this library extends (config 3, GF(2^16)) as a
    resident square: its data root equals tests/golden/k512.json's, and share
    proofs across the square validate against it (the proof nodes and aunts come from every cached level); a
    subtree walk of row 1 023 (a Q2 | Q3 row) equals the tree
    over that row's cells."""
    import json
    import os
    from celestia_da import testfactory
    from test_share_proof_validate import to_dict
    k = 512
    want = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "k512.json")))["squares"]["0"]
    ods = testfactory.random_square(k, 0)
    sq = gpr.ResidentSquare(ods)
    try:
        rows, _, root = sq.dah()
        assert root.hex() == want["data_root"]
        shares = ods.reshape(-1, 512)
        # every share of a random square has its own namespace, so the proofs
        # are of single shares (Validate needs one namespace): first / last of
        # rows, the middle, the last ODS share
        for s in (0, 5, k - 1, k, 3 * k + 100, k * k // 2 + 17, k * k - 1):
            p = sq.share_proof(bytes(shares[s][:29]), s, s + 1)
            assert opr.share_proof_validate(to_dict(p), root) is None, s
            assert p.data == [bytes(shares[s])]
        eds_row = sq.eds()[2 * k - 1]
        leaves = pyref.erasured_leaves([bytes(c) for c in eds_row], k, 2 * k - 1)
        walk = [True, False, True, True, False, False, True, False, True]
        assert sq.subtree_root(2 * k - 1, walk) == opr.walk_subtree_root(leaves, walk)
        assert sq.subtree_root(2 * k - 1, []) == rows[2 * k - 1]
    finally:
        sq.close()
