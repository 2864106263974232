"""App-level DA entry points (celestia_da.app): ExtendBlock / IsEmptyBlock
(app/extend_block.go:13-32) and the DA checks of ProcessProposal
(app/process_proposal.go:122-152) with the reference's rejection reasons.

Pinned by mainnet block 408 (its header DataHash and square size, and the
ODS decoded from the reference fixture x/blob/test/testdata/block_response.json).
"""
import numpy as np
import pytest

from celestia_da import app, blobfactory, da
from celestia_da import square as gsq
from test_square import block408, block408_ods


def test_versioned_consts():
    for v in (1, 2, app.LATEST_VERSION):
        assert app.square_size_upper_bound(v) == 128
        assert app.subtree_root_threshold(v) == 64


def test_is_empty_block():
    assert app.is_empty_block([])
    assert not app.is_empty_block([b"x"])


def _bad_block():
    rng = np.random.default_rng(3)
    return blobfactory.random_block(12, 1, 2) + [blobfactory.normal_tx(rng, 100)]


@pytest.mark.gpu
def test_extend_block_block408(ctx):
    txs, k, data_hash = block408()
    eds = app.extend_block(txs, ctx=ctx)
    assert eds.width() == 2 * k
    assert eds.array()[:k, :k].tobytes() == block408_ods()
    dah = da.new_data_availability_header(eds)
    assert dah.hash() == data_hash
    # the same EDS and roots as Construct then ExtendShares as two calls
    ref = da.extend_shares(list(gsq.construct(txs)))
    assert np.array_equal(ref.array(), eds.array())
    assert ref.row_roots() == eds.row_roots() and ref.col_roots() == eds.col_roots()


@pytest.mark.gpu
def test_extend_block_errors_and_empty(ctx):
    from celestia_da import SquareError
    with pytest.raises(SquareError, match="normal transaction at index 3"):
        app.extend_block(_bad_block(), ctx=ctx)
    eds = app.extend_block([], ctx=ctx)
    assert eds.width() == 2
    assert da.new_data_availability_header(eds).hash() == da.min_data_availability_header().hash()


@pytest.mark.gpu
def test_process_proposal_da_reasons(ctx):
    txs, k, data_hash = block408()
    v = app.process_proposal_da(txs, k, data_hash, ctx=ctx)
    assert v.accept and v.reason is None and v.data_root == data_hash
    v = app.process_proposal_da(txs, 2 * k, data_hash, ctx=ctx)
    assert not v.accept and v.reason == "proposed square size differs from calculated square size"
    wrong = bytes(32)
    v = app.process_proposal_da(txs, k, wrong, ctx=ctx)
    assert not v.accept
    assert v.reason == (f"proposed data root {'00' * 32} differs from calculated data root "
                        f"{data_hash.hex().upper()}")
    v = app.process_proposal_da(_bad_block(), 8, wrong, ctx=ctx)
    assert not v.accept and v.reason.startswith(
        "failure to compute data square from transactions: normal transaction at index 3")


@pytest.mark.gpu
def test_process_proposals_da_batch_equals_per_block(ctx):
    txs, k, data_hash = block408()
    blocks = [txs, _bad_block(), blobfactory.full_block(5, 64), [], txs, blobfactory.full_block(6, 128)]
    sizes, hashes = [], []
    for i, b in enumerate(blocks):
        try:
            kk, _, _, _, root, _ = gsq.construct_extend_dah(b, ctx=ctx)
        except Exception:
            kk, root = 8, bytes(32)
        sizes.append(kk + (i == 4))           # block 4: a wrong proposed size
        hashes.append(root if i != 2 else bytes(32))   # block 2: a wrong data hash
    got = app.process_proposals_da(blocks, sizes, hashes, ctx=ctx)
    want = [app.process_proposal_da(b, s, h, ctx=ctx) for b, s, h in zip(blocks, sizes, hashes)]
    assert got == want
    assert [v.accept for v in got] == [True, False, False, True, False, True]


@pytest.mark.gpu
def test_prepare_then_process(ctx):
    """A proposal built by prepare_proposal_da is accepted by
    process_proposal_da (the round trip every honest block takes); Build
    drops what does not fit and reorders normal txs first."""
    rng = np.random.default_rng(9)
    txs = blobfactory.random_block(21, 3, 20, (1, 2), (1, 20000)) + [blobfactory.normal_tx(rng, 300)]
    bd = app.prepare_proposal_da(txs, ctx=ctx)
    assert bd.txs[0] is txs[0] and txs[-1] in bd.txs[:4]
    sq, kept = gsq.build(txs, 128, 64, ctx=ctx)
    assert bd.txs == kept and bd.square_size == sq.size()
    v = app.process_proposal_da(bd.txs, bd.square_size, bd.hash, ctx=ctx)
    assert v.accept, v.reason
    big = blobfactory.random_block(11, 2, 400, (1, 2), (20000, 60000))
    bd = app.prepare_proposal_da(big, ctx=ctx)
    assert bd.square_size == 128 and 0 < len(bd.txs) < len(big)
    assert app.process_proposal_da(bd.txs, 128, bd.hash, ctx=ctx).accept


@pytest.mark.gpu
def test_process_proposal_mutations(ctx):
    """TestProcessProposal's cases a DA check decides (app/test/process_proposal_test.go:92-333):
    PrepareProposal's block data is mutated, then ProcessProposal judges it
    against the header DataHash.  (Signature, nonce and decoding cases need
    the ante handler and state: out of scope.)"""
    txs = blobfactory.random_block(31, 2, 4, (1, 2), (100, 5000))     # [normal, normal, blob txs...]
    bd = app.prepare_proposal_da(txs, ctx=ctx)
    assert bd.txs == txs

    def judge(t, size=None, h=None):
        return app.process_proposal_da(t, bd.square_size if size is None else size, bd.hash if h is None else h,
                                       ctx=ctx)

    assert judge(bd.txs).accept                                               # valid untouched data
    data_root_reason = "proposed data root " + bd.hash.hex().upper() + " differs from calculated data root"
    for name, mutated in [("removed first blob tx", bd.txs[:2] + bd.txs[3:]),
                          ("added an extra blob tx", bd.txs + [bd.txs[3]]),
                          ("swap blobTxs", bd.txs[:2] + [bd.txs[3], bd.txs[4], bd.txs[2]] + bd.txs[5:])]:
        v = judge(mutated)   # the reference expects REJECT; which check fires depends on the square it gives
        assert not v.accept and (v.reason.startswith(data_root_reason) or
                                 v.reason == "proposed square size differs from calculated square size"), name
    # incorrectly sorted; a normal tx after a PFB: square.Construct rejects the order
    v = judge(bd.txs[:1] + [bd.txs[2], bd.txs[1]] + bd.txs[3:])
    assert not v.accept and v.reason.startswith("failure to compute data square from transactions: normal transaction")
    # tampered sequence start: the header commits to share 1 with its
    # sequence-start bit flipped (shares.Builder.FlipSequenceStart), which the
    # honest square does not have
    sq = list(gsq.construct(bd.txs, ctx=ctx))
    sq[1] = sq[1][:29] + bytes([sq[1][29] ^ 1]) + sq[1][30:]
    tampered = da.new_data_availability_header(da.extend_shares(sq)).hash()
    assert tampered != bd.hash
    v = judge(bd.txs, h=tampered)
    assert not v.accept and v.reason.startswith("proposed data root " + tampered.hex().upper())


def test_max_effective_square_size():
    """App.MaxEffectiveSquareSize (app/square_size.go:9-23)."""
    assert app.max_effective_square_size() == 128
    assert app.max_effective_square_size(64) == 64
    assert app.max_effective_square_size(256) == 128
    assert app.max_effective_square_size(128, height=1) == app.DEFAULT_GOV_MAX_SQUARE_SIZE == 64


# TestPrepareProposalConsistency's tx shapes (app/test/fuzz_abci_test.go:40-50):
# (name, blob txs, blobs per tx, blob bytes), scaled where the reference's
# count would only be dropped by Build anyway, plus its send txs (:98-108)
CONSISTENCY_SHAPES = [
    ("many small single share single blob transactions", 1000, 1, 400),
    ("one hundred normal sized single blob transactions", 100, 1, 400000),
    ("many single share multi-blob transactions", 200, 100, 400),
    ("one hundred normal sized multi-blob transactions", 30, 4, 400000),
]


@pytest.mark.gpu
@pytest.mark.parametrize("gov_max", [64, 128])
def test_prepare_proposal_consistency(ctx, gov_max):
    """Every block PrepareProposal builds is accepted by ProcessProposal
    (fuzz_abci_test.go:26-137), for the default governance square size (64)
    and the hard maximum, one at a time and as one replay batch."""
    prepared = []
    for i, (name, n, per_tx, size) in enumerate(CONSISTENCY_SHAPES):
        txs = blobfactory.random_block(100 + i, 100, n, (per_tx, per_tx), (size, size))
        bd = app.prepare_proposal_da(txs, ctx=ctx, gov_max_square_size=gov_max)
        assert 1 <= bd.square_size <= gov_max and bd.txs, name
        v = app.process_proposal_da(bd.txs, bd.square_size, bd.hash, ctx=ctx, gov_max_square_size=gov_max)
        assert v.accept, (name, v.reason)
        prepared.append(bd)
    got = app.process_proposals_da([b.txs for b in prepared], [b.square_size for b in prepared],
                                   [b.hash for b in prepared], ctx=ctx, gov_max_square_size=gov_max)
    assert all(v.accept for v in got), [v.reason for v in got]
