"""Transaction inclusion proofs: proof.NewTxInclusionProof (pkg/proof/proof.go:22-57)
over go-square's builder.FindTxShareRange.

CPU: cda_square_tx_share_range (csrc/square_plan.cpp, the compact-share
splitters' recorded ranges) against the oracle's restatement
(oracle/square.py find_tx_share_range) on every tx of several blocks --
mainnet block 408, the reference test's shape (50 normal txs of 500 B, then
50 blob txs with one 500-B blob: pkg/proof/proof_test.go:27-96), repeated
txs (the splitters key ranges by tx hash) and txs that end exactly on a
share boundary -- and the reference's error cases.
GPU: the proofs of the indexes the reference test proves (first / last
normal, first / last blob tx) and of every tx of block 408 verify against the
oracle's row roots and data root (block 408: its header DataHash), and cover
exactly the shares of the tx's compact range.
"""
import ctypes as C

import numpy as np
import pytest

import proofs as opr
import pyref
import square as osq
from celestia_da import CdaError, SquareError, _lib, blobfactory
from celestia_da import proof as gpr
from celestia_da import square as gsq
from test_proofs import oracle_eds
from test_share_proof_validate import to_dict
from test_square import block408


def _reference_shape_block(seed=3):
    rng = np.random.default_rng(seed)
    normal = [blobfactory.normal_tx(rng, 500) for _ in range(50)]
    blob_txs = blobfactory.random_block(seed, 0, 50, (1, 1), (500, 500))
    return normal + blob_txs


def _blocks():
    rng = np.random.default_rng(11)
    dup = [blobfactory.normal_tx(rng, 300) for _ in range(3)]
    return {
        "block408": block408()[0],
        "reference_shape": _reference_shape_block(),
        "normal_only": blobfactory.random_block(5, 30, 0),
        "repeated": [dup[0], dup[1], dup[0], dup[2], dup[0]],
        # 472 + 2 varint bytes fill the first share's 474, 476 + 2 a continuation's 478
        "share_boundaries": [bytes([7]) * 472, bytes([8]) * 476, bytes([9]) * 10, bytes([1]) * 1000],
        "many_blobs": blobfactory.random_block(8, 4, 40, (1, 3), (1, 9000), 3),
    }


def _c_range(txs, i):
    buf, off = gsq._flatten(txs)
    s, e, p = C.c_uint32(), C.c_uint32(), C.c_int()
    L = _lib.load()
    rc = L.cda_square_tx_share_range(None, gsq.ptr(buf), gsq._u64p(off), len(txs), 128, 64, i, C.byref(s), C.byref(e),
                                     C.byref(p))
    if rc != _lib.CDA_OK:
        return "error", L.cda_last_error(None).decode()
    return s.value, e.value, bool(p.value)


@pytest.mark.parametrize("name", list(_blocks()))
def test_tx_share_range_matches_oracle(name):
    txs = _blocks()[name]
    for i in range(len(txs) + 1):
        try:
            want = osq.find_tx_share_range(txs, i)
        except ValueError as e:
            want = ("error", str(e))
        assert _c_range(txs, i) == want, (name, i)


def test_tx_share_range_semantics():
    b = _blocks()
    # repeated txs report the last copy's range
    r = [_c_range(b["repeated"], i) for i in range(5)]
    assert r[0] == r[2] == r[4] and r[0] != r[1]
    # exact fills: each tx owns one share
    assert [_c_range(b["share_boundaries"], i)[:2] for i in range(3)] == [(0, 1), (1, 2), (2, 3)]
    # the reference shape: normal txs in the tx namespace, blob txs in the PFB namespace after them
    txs = b["reference_shape"]
    s49, e49, ns49 = gpr.tx_share_range(txs, 49)
    s50, e50, ns50 = gpr.tx_share_range(txs, 50)
    assert ns49 == gpr.TX_NAMESPACE and ns50 == gpr.PAY_FOR_BLOB_NAMESPACE
    assert e49 <= s50 + 1 and s50 >= 1


def test_tx_inclusion_proof_errors():
    with pytest.raises(CdaError, match="txIndex 0 out of bounds"):
        gpr.new_tx_inclusion_proof([], 0)
    txs = _reference_shape_block()
    with pytest.raises(CdaError, match="txIndex 100 out of bounds"):
        gpr.new_tx_inclusion_proof(txs, 100)
    rng = np.random.default_rng(3)
    bad = blobfactory.random_block(12, 1, 2) + [blobfactory.normal_tx(rng, 100)]
    with pytest.raises(SquareError, match="normal transaction at index 3"):
        gpr.tx_share_range(bad, 0)


def _verify(txs, idx, data_hash=None):
    """NewTxInclusionProof for each index, checked against the oracle."""
    shares, k, _, _ = osq.builder(txs, 128, 64, "construct")
    ods = np.frombuffer(b"".join(shares), dtype=np.uint8).reshape(-1, 512).copy()
    eds, rows, cols, root = oracle_eds(ods, k)
    if data_hash is not None:
        assert root == data_hash
    items = rows + cols
    for i in idx:
        s, e, pfb = osq.find_tx_share_range(txs, i)
        ns = osq.PFB_NS if pfb else osq.TX_NS
        p = gpr.new_tx_inclusion_proof(txs, i)
        assert opr.share_proof_validate(to_dict(p), root) is None
        assert bytes([p.namespace_version]) + p.namespace_id == ns
        assert p.data == [shares[j] for j in range(s, e)]
        assert all(d[:29] == ns for d in p.data)
        r0, r1 = s // k, (e - 1) // k
        assert (p.row_proof.start_row, p.row_proof.end_row) == (r0, r1)
        for q, r in enumerate(range(r0, r1 + 1)):
            sp = p.share_proofs[q]
            leaves = pyref.erasured_leaves([bytes(c) for c in eds[r]], k, r)
            assert opr.nmt_verify_range(rows[r], sp.nodes, sp.start, sp.end, 2 * k, leaves[sp.start:sp.end])
            rp = p.row_proof.proofs[q]
            assert opr.rfc_verify(root, rp.total, rp.index, rp.leaf_hash, rp.aunts)
            assert p.row_proof.row_roots[q] == items[r]


@pytest.mark.gpu
def test_tx_inclusion_proofs_reference_shape(ctx):
    _verify(_reference_shape_block(), [0, 49, 50, 99])


@pytest.mark.gpu
def test_tx_inclusion_proofs_block408(ctx):
    txs, _, data_hash = block408()
    _verify(txs, range(len(txs)), data_hash)


@pytest.mark.gpu
def test_tx_inclusion_proofs_boundaries_and_repeats(ctx):
    b = _blocks()
    _verify(b["share_boundaries"], range(4))
    _verify(b["repeated"], range(5))


def _all_shares_block(seed=17):
    """TestAllSharesInclusionProof's block (pkg/proof/proof_test.go:241-268):
    testfactory.GenerateRandomTxs(243, 500) -- 243 normal txs of 500 B."""
    rng = np.random.default_rng(seed)
    return [blobfactory.normal_tx(rng, 500) for _ in range(243)]


def test_all_shares_block_layout():
    """The reference asserts the square holds 256 shares, all in the tx
    namespace (ParseNamespace over [0, 256))."""
    shares, k, _, _ = osq.builder(_all_shares_block(), 128, 64, "construct")
    assert (len(shares), k) == (256, 16)
    assert all(s[:29] == osq.TX_NS for s in shares)
    s, e, pfb = osq.find_tx_share_range(_all_shares_block(), 242)
    assert (e, pfb) == (256, False)


@pytest.mark.gpu
def test_all_shares_inclusion_proof(ctx):
    """NewShareInclusionProof(square, TxNamespace, [0, 256)) validates against
    the data root (proof_test.go:241-268)."""
    shares, k, _, _ = osq.builder(_all_shares_block(), 128, 64, "construct")
    ods = np.frombuffer(b"".join(shares), dtype=np.uint8).reshape(-1, 512).copy()
    _, rows, _, root = oracle_eds(ods, k)
    p = gpr.new_share_inclusion_proof(ods, osq.TX_NS, 0, 256)
    assert opr.share_proof_validate(to_dict(p), root) is None
    assert (p.row_proof.start_row, p.row_proof.end_row) == (0, k - 1)
    assert p.data == shares and p.row_proof.row_roots == rows[:k]
    bad = to_dict(p)
    bad["data"] = [bytes(512)] + bad["data"][1:]
    assert opr.share_proof_validate(bad, root) is not None


def _share_proof_block():
    """TestNewShareInclusionProof's block (pkg/proof/proof_test.go:98-107): 50
    random txs of 500 B, then three blob txs with one 500-B blob each in ns1,
    ns2, ns3 (appns.MustNewV0 of ten 0x01 / 0x02 / 0x03 bytes)."""
    rng = np.random.default_rng(23)
    txs = [blobfactory.normal_tx(rng, 500) for _ in range(50)]
    for b in (1, 2, 3):   # signed PFB txs of ~450 B: three compact shares, as in the reference's square
        inner = rng.integers(0, 256, 450, dtype=np.uint8).tobytes()
        txs.append(blobfactory.blob_tx(inner, [(b"\x00" * 18 + bytes([b]) * 10,
                                                 rng.integers(0, 256, 500, dtype=np.uint8).tobytes())]))
    return txs


NS = {b: b"\x00" * 19 + bytes([b]) * 10 for b in (1, 2, 3)}
# (name, start, end, namespace or None when ParseNamespace must fail), proof_test.go:122-209
SHARE_PROOF_CASES = [
    ("negative starting share", -1, 99, None),
    ("negative ending share", 0, -99, None),
    ("ending share lower than starting share", 1, 0, None),
    ("ending share is equal to the starting share", 1, 1, None),
    ("ending share higher than number of shares available in square size of 32", 0, 4097, None),
    ("1 transaction share", 0, 1, gpr.TX_NAMESPACE),
    ("10 transaction shares", 0, 10, gpr.TX_NAMESPACE),
    ("53 transaction shares", 0, 53, gpr.TX_NAMESPACE),
    ("shares from different namespaces", 48, 55, None),
    ("shares from PFB namespace", 53, 55, gpr.PAY_FOR_BLOB_NAMESPACE),
    ("blob shares for first namespace", 56, 58, NS[1]),
    ("blob shares for third namespace", 60, 62, NS[3]),
]


def test_parse_namespace_cases():
    """ParseNamespace over the reference test's square shape: the same share
    indexes hold the same namespaces (53 tx shares, the PFB shares, 2-share
    blobs at 56 and 60), and the error cases fail with querier.go's texts."""
    shares, k, _, _ = osq.builder(_share_proof_block(), 128, 64, "construct")
    assert k == 8
    for name, s, e, ns in SHARE_PROOF_CASES:
        if ns is None:
            with pytest.raises(ValueError):
                gpr.parse_namespace(shares, s, e)
        else:
            assert gpr.parse_namespace(shares, s, e) == ns, name
    with pytest.raises(ValueError, match="start share -1 should be positive"):
        gpr.parse_namespace(shares, -1, 99)
    with pytest.raises(ValueError, match="end share 0 cannot be lower or equal to the starting share 1"):
        gpr.parse_namespace(shares, 1, 0)
    with pytest.raises(ValueError, match="end share 4097 is higher than block shares 64"):
        gpr.parse_namespace(shares, 0, 4097)
    with pytest.raises(ValueError) as e:
        gpr.parse_namespace(shares, 48, 55)
    assert str(e.value) == ("shares range contain different namespaces at index 5: {0 [" + " ".join(["0"] * 27) +
                            " 1]} and {0 [" + " ".join(["0"] * 27) + " 4]} ")


@pytest.mark.gpu
def test_new_share_inclusion_proof_cases(ctx):
    """TestNewShareInclusionProof (proof_test.go:98-238): every range
    ParseNamespace accepts gets a GPU proof that validates against the data
    root."""
    shares, k, _, _ = osq.builder(_share_proof_block(), 128, 64, "construct")
    ods = np.frombuffer(b"".join(shares), dtype=np.uint8).reshape(-1, 512).copy()
    _, _, _, root = oracle_eds(ods, k)
    sq = gpr.ResidentSquare(ods)
    try:
        for name, s, e, ns in SHARE_PROOF_CASES:
            if ns is None:
                continue
            p = sq.share_proof(gpr.parse_namespace(shares, s, e), s, e)
            assert opr.share_proof_validate(to_dict(p), root) is None, name
            assert p.data == shares[s:e]
    finally:
        sq.close()


def test_query_tx_inclusion_proof_rejects_negative_values():
    """TestQueryTxInclusionProofRejectsNegativeValues (proof_test.go:270-287)
    and the querier's other index checks (querier.go:29-40)."""
    with pytest.raises(ValueError, match="negative") as e:
        gpr.query_tx_inclusion_proof(["-2"], [])
    assert str(e.value) == 'path[0] element: "-2" produced a negative value: -2'
    with pytest.raises(ValueError, match="expected query path length: 1 actual: 2 "):
        gpr.query_tx_inclusion_proof(["1", "2"], [])
    with pytest.raises(ValueError, match='parsing "x1": invalid syntax'):
        gpr.query_tx_inclusion_proof(["x1"], [])
    with pytest.raises(ValueError, match="value out of range"):
        gpr.query_tx_inclusion_proof([str(1 << 63)], [])
    with pytest.raises(CdaError, match="txIndex -1 is negative"):
        gpr.new_tx_inclusion_proof([b"x"], -1)


def test_query_share_inclusion_proof_path_errors():
    """QueryShareInclusionProof's path checks (querier.go:72-84) and the
    ParseNamespace texts it passes through."""
    with pytest.raises(ValueError, match="expected query path length: 2 actual: 1 "):
        gpr.query_share_inclusion_proof(["3"], [])
    with pytest.raises(ValueError, match='parsing "a": invalid syntax'):
        gpr.query_share_inclusion_proof(["a", "5"], [])


@pytest.mark.gpu
def test_query_share_inclusion_proof(ctx):
    """custom/shareInclusionProof/56/58 over the block of
    TestNewShareInclusionProof: ns1's blob shares, validated."""
    txs = _share_proof_block()
    shares, k, _, _ = osq.builder(txs, 128, 64, "construct")
    ods = np.frombuffer(b"".join(shares), dtype=np.uint8).reshape(-1, 512).copy()
    _, _, _, root = oracle_eds(ods, k)
    p = gpr.query_share_inclusion_proof(["56", "58"], txs)
    assert bytes([p.namespace_version]) + p.namespace_id == NS[1]
    assert opr.share_proof_validate(to_dict(p), root) is None
    with pytest.raises(ValueError, match="shares range contain different namespaces"):
        gpr.query_share_inclusion_proof(["48", "55"], txs)
    with pytest.raises(ValueError, match="start share -1 should be positive"):   # after Construct, as in Go
        gpr.query_share_inclusion_proof(["-1", "5"], txs)
