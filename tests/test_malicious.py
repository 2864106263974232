"""Unordered squares, as the reference's fraud tooling builds them
(test/util/malicious: BlindTree, tree.go:18-58, pushes with ForceAddLeaf and
hashes with the malicious hasher, hasher.go:161-310, which checks no
namespace order).

TestOutOfOrderNMT (app_test.go:19-60) on the oracle: the blind tree's root
equals the honest tree's on ordered data, and on shuffled data it is a 90-byte
root that differs, where the honest tree fails with ErrInvalidPushOrder.

GPU: the library's answer for an unordered square is the honest one --
CDA_ERR_PUSH_ORDER with nmt's message, which rejects the block in
ProcessProposal (app/process_proposal.go:144-147) -- and what it still writes
is the malicious package's square: the EDS of malicious.ExtendShares
(tree.go:60-71, the same codec) and the row / column roots and data root of
NewDataAvailabilityHeader over BlindTrees (the hashing never depends on the
order check), in the single-square and the batch entry points alike.
"""
import ctypes as C

import numpy as np
import pytest

import pyref
from celestia_da import da, malicious, testfactory
from celestia_da._lib import CDA_ERR_PUSH_ORDER, ptr


def _shuffled(cells, seed):
    rng = np.random.default_rng(seed)
    out = list(cells)
    for i in range(len(out)):          # the reference test's swap loop
        j = int(rng.integers(len(out)))
        out[i], out[j] = out[j], out[i]
    return out


def test_out_of_order_nmt():
    k = 64
    data = [bytes(c) for c in testfactory.random_namespaced_shares(64, 7)]
    good = pyref.axis_root(data, k, 0)
    assert pyref.axis_root(data, k, 0, blind=True) == good
    bad = _shuffled(data, 1)
    assert bad != data
    with pytest.raises(pyref.PushOrderError):
        pyref.axis_root(bad, k, 0)
    root = pyref.axis_root(bad, k, 0, blind=True)
    assert len(root) == 90 and root != good


def _unordered_square(k, seed):
    ods = testfactory.random_square(k, seed).reshape(k, k, 512).copy()
    ods[1, [0, 3]] = ods[1, [3, 0]]                # row 1 and columns 0 / 3 out of order
    return ods


def test_blind_dah_of_unordered_square():
    """The blind DAH exists for an unordered square and differs from every
    ordered square's; the honest one fails at the first Q0 tree."""
    k = 4
    ods = _unordered_square(k, 3)
    eds = pyref.extend_square(ods)
    with pytest.raises(pyref.PushOrderError):
        pyref.dah_from_eds(eds)
    rows, cols, root = pyref.dah_from_eds(eds, blind=True)
    assert len(rows) == len(cols) == 2 * k and all(len(r) == 90 for r in rows + cols)
    _, _, good_root = pyref.dah_from_eds(pyref.extend_square(testfactory.random_square(k, 3).reshape(k, k, 512)))
    assert root != good_root


@pytest.mark.gpu
@pytest.mark.parametrize("k", [4, 16])
def test_unordered_square_rejected_eds_written(ctx, k):
    ods = _unordered_square(k, 5)
    W = 2 * k
    eds = np.zeros(W * W * 512, dtype=np.uint8)
    rows = np.empty(W * 90, dtype=np.uint8)
    cols = np.empty(W * 90, dtype=np.uint8)
    root = np.empty(32, dtype=np.uint8)
    rc = ctx.lib.cda_extend_dah(ctx.h, ptr(np.ascontiguousarray(ods)), k * k, ptr(eds), ptr(rows), ptr(cols),
                                ptr(root))
    assert rc == CDA_ERR_PUSH_ORDER
    msg = ctx.lib.cda_last_error(ctx.h).decode()
    with pytest.raises(pyref.PushOrderError) as want:
        pyref.dah_from_eds(pyref.extend_square(ods))
    assert msg == str(want.value)
    want_eds = pyref.extend_square(ods)
    assert np.array_equal(eds.reshape(W, W, 512), want_eds)
    r, c, d = pyref.dah_from_eds(want_eds, blind=True)
    assert rows.tobytes() == b"".join(r) and cols.tobytes() == b"".join(c) and root.tobytes() == d
    # the Python mirror of malicious.ExtendShares + NewDataAvailabilityHeader
    m_eds, dah = malicious.extend_shares_dah(list(ods.reshape(k * k, 512)))
    assert np.array_equal(m_eds, want_eds)
    assert (dah.row_roots, dah.column_roots, dah.hash()) == (r, c, d)
    # ... equal to the honest header on an ordered square
    good = testfactory.random_square(k, 5).reshape(k * k, 512)
    _, gd = malicious.extend_shares_dah(list(good))
    hd = da.new_data_availability_header(da.extend_shares(list(good)))
    assert (gd.row_roots, gd.column_roots, gd.hash()) == (hd.row_roots, hd.column_roots, hd.hash())


@pytest.mark.gpu
def test_batch_with_one_unordered_square(ctx):
    """cda_extend_dah_batch: only the unordered square's status is set; its
    roots are the blind ones, the others the honest ones."""
    k, n = 8, 3
    ods = np.stack([testfactory.random_square(k, 20 + i).reshape(k, k, 512) for i in range(n)])
    ods[1] = _unordered_square(k, 21)
    W = 2 * k
    rows = np.empty(n * W * 90, dtype=np.uint8)
    cols = np.empty(n * W * 90, dtype=np.uint8)
    roots = np.empty(n * 32, dtype=np.uint8)
    status = np.empty(n, dtype=np.int32)
    rc = ctx.lib.cda_extend_dah_batch(ctx.h, ptr(np.ascontiguousarray(ods)), k, n, None, ptr(rows), ptr(cols),
                                      ptr(roots), status.ctypes.data_as(C.POINTER(C.c_int32)))
    assert rc == CDA_ERR_PUSH_ORDER and status.tolist() == [0, CDA_ERR_PUSH_ORDER, 0]
    for i in range(n):
        r, c, d = pyref.dah_from_eds(pyref.extend_square(ods[i]), blind=(i == 1))
        assert rows[i * W * 90:(i + 1) * W * 90].tobytes() == b"".join(r)
        assert cols[i * W * 90:(i + 1) * W * 90].tobytes() == b"".join(c)
        assert roots[32 * i:32 * (i + 1)].tobytes() == d
