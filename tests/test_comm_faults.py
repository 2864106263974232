"""Error paths of the library's RCCL split (cda_extend_dah_split, config 5).

VERDICT r2 item 7 / ADVICE r2: a failing RCCL call must close its group
(ncclGroupEnd), abort the communicator and return a distinct code
(CDA_ERR_COMM); a local failure must not leave the peers blocked (the rank
stays in every collective and poisons the push-order word); an allocation
failure on any rank must fail every rank before any data-path collective.
World size 1 on the test box's single GPU (RCCL self send/recv), each fault
forced through CDA_COMM_FAULT (read by the library at every split call); after
every fault a clean call -- on the same communicator, or on a fresh one when
it was aborted -- must match the single-GPU path.  Reference analogue: the
ProcessProposal rejection path (app/process_proposal.go:139-147) must see an
error, never a hang or an abort.
"""
import os

import pytest

import knobs

pytestmark = pytest.mark.gpu


def _clean_split_matches(ctx, c, d_ods, k):
    import torch
    from celestia_da import dist as cdist
    dev = d_ods.device
    block, (rows, cols, root, err) = cdist.extend_dah_split_rccl(c, d_ods, k, 0, 1)
    torch.cuda.synchronize()
    assert int(err.item()) == 0xFFFFFFFF
    W = 2 * k
    e = torch.empty(W * W * 512, dtype=torch.uint8, device=dev)
    r1 = torch.empty(W * 90, dtype=torch.uint8, device=dev)
    c1 = torch.empty(W * 90, dtype=torch.uint8, device=dev)
    g1 = torch.empty(32, dtype=torch.uint8, device=dev)
    ctx.extend_dah_device(d_ods.data_ptr(), k, 1, e.data_ptr(), r1.data_ptr(), c1.data_ptr(), g1.data_ptr(),
                          None, torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(block.view(-1), e)
    assert torch.equal(rows.view(-1), r1) and torch.equal(cols.view(-1), c1) and torch.equal(root, g1)


def _split_rc(c, d_ods, k, want_err_word=None):
    """Raw cda_extend_dah_split call: (rc, message, reduced err word)."""
    import torch
    dev = d_ods.device
    W = 2 * k
    block = torch.empty((W, W, 512), dtype=torch.uint8, device=dev)
    err = torch.empty((1,), dtype=torch.int32, device=dev)
    rows = torch.empty((W, 90), dtype=torch.uint8, device=dev)
    cols = torch.empty((W, 90), dtype=torch.uint8, device=dev)
    root = torch.empty((32,), dtype=torch.uint8, device=dev)
    rc = c.lib.cda_extend_dah_split(c.h, d_ods.data_ptr(), k, block.data_ptr(), rows.data_ptr(), cols.data_ptr(),
                                    root.data_ptr(), err.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    msg = c.lib.cda_last_error(c.h).decode()
    torch.cuda.synchronize()
    return rc, msg, int(err.item()) & 0xFFFFFFFF


@pytest.fixture
def comm_setup():
    import torch
    from celestia_da import _lib, testfactory
    k = 16
    dev = torch.device("cuda", 0)
    d_ods = torch.from_numpy(testfactory.random_square(k, 9)).to(dev)
    c = _lib.Context(0, lib_path=knobs.lib_path_for_tests())   # CDA_COMM_FAULT: test build only
    c.comm_init(0, 1, _lib.comm_unique_id())
    yield c, d_ods, k
    os.environ.pop("CDA_COMM_FAULT", None)
    c.comm_destroy()
    c.close()


def test_comm_size_reports_the_communicator(ctx, comm_setup):
    """cda_comm_size: the rank and rank count RCCL formed (what bench.py
    reports as config 5's communicator_ranks); no communicator -> error."""
    from celestia_da import CdaError, _lib
    c, _, _ = comm_setup
    assert c.comm_size() == (0, 1)
    c.comm_destroy()
    with pytest.raises(CdaError, match="cda_comm_init"):
        c.comm_size()
    c.comm_init(0, 1, _lib.comm_unique_id())
    assert c.comm_size() == (0, 1)


@pytest.mark.parametrize("where", ["gather", "a2a_or_gather"])
def test_rccl_failure_closes_group_aborts_and_recovers(ctx, comm_setup, where):
    """A failed RCCL call inside a group: CDA_ERR_COMM, the communicator is
    gone (the next split says so), and a fresh communicator works."""
    from celestia_da import _lib
    c, d_ods, k = comm_setup
    _clean_split_matches(ctx, c, d_ods, k)
    # world 1 has no all-to-all group: "a2a" must leave it untouched, the
    # gather group still fails
    os.environ["CDA_COMM_FAULT"] = "gather" if where == "gather" else "a2a"
    rc, msg, _ = _split_rc(c, d_ods, k)
    if where == "gather":
        assert rc == _lib.CDA_ERR_COMM, (rc, msg)
        assert "gather" in msg and "aborted" in msg
        os.environ.pop("CDA_COMM_FAULT")
        rc2, msg2, _ = _split_rc(c, d_ods, k)
        assert rc2 == _lib.CDA_ERR_INVALID and "cda_comm_init" in msg2
        c.comm_init(0, 1, _lib.comm_unique_id())
    else:
        assert rc == _lib.CDA_OK, (rc, msg)
        os.environ.pop("CDA_COMM_FAULT")
    _clean_split_matches(ctx, c, d_ods, k)


def test_local_failure_poisons_and_keeps_communicator(ctx, comm_setup):
    """A local failure (the column stage) keeps the rank in the remaining
    collectives: the call returns the local error, the MIN-reduced push-order
    word is 0 (never a valid violation word), and the communicator is still
    usable for the next call."""
    from celestia_da import _lib
    c, d_ods, k = comm_setup
    os.environ["CDA_COMM_FAULT"] = "local"
    rc, msg, word = _split_rc(c, d_ods, k)
    assert rc == _lib.CDA_ERR_DEVICE and "injected" in msg, (rc, msg)
    assert word == 0
    os.environ.pop("CDA_COMM_FAULT")
    _clean_split_matches(ctx, c, d_ods, k)


def test_allocation_agreement_fails_every_rank_cleanly(ctx, comm_setup):
    """Scratch is sized when k changes, then one agreement all-reduce: a rank
    that cannot allocate makes the call fail with CDA_ERR_OOM before any
    data-path collective, and the communicator stays usable."""
    import torch
    from celestia_da import _lib, testfactory
    c, d_ods, k = comm_setup
    _clean_split_matches(ctx, c, d_ods, k)
    k2 = 32
    d2 = torch.from_numpy(testfactory.random_square(k2, 10)).to(d_ods.device)
    os.environ["CDA_COMM_FAULT"] = "alloc"
    rc, msg, _ = _split_rc(c, d2, k2)
    assert rc == _lib.CDA_ERR_OOM and "allocation" in msg, (rc, msg)
    os.environ.pop("CDA_COMM_FAULT")
    _clean_split_matches(ctx, c, d2, k2)


def test_null_rank0_outputs_fail_after_collectives(ctx, comm_setup):
    """Rank 0 without output buffers: CDA_ERR_INVALID, returned after the
    rank took part in every collective (its peers are not left blocked);
    the communicator stays usable."""
    import torch
    from celestia_da import _lib
    c, d_ods, k = comm_setup
    dev = d_ods.device
    err = torch.empty((1,), dtype=torch.int32, device=dev)
    rc = c.lib.cda_extend_dah_split(c.h, d_ods.data_ptr(), k, None, None, None, None, err.data_ptr(),
                                    torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    assert rc == _lib.CDA_ERR_INVALID
    assert int(err.item()) == 0
    _clean_split_matches(ctx, c, d_ods, k)


def test_comm_abort_without_lock(ctx, comm_setup):
    """cda_comm_abort releases the communicator (a watchdog's way out)."""
    from celestia_da import _lib
    c, d_ods, k = comm_setup
    c.comm_abort()
    rc, msg, _ = _split_rc(c, d_ods, k)
    assert rc == _lib.CDA_ERR_INVALID and "cda_comm_init" in msg
    c.comm_init(0, 1, _lib.comm_unique_id())
    _clean_split_matches(ctx, c, d_ods, k)



def test_peer_failure_fails_rank0(ctx, comm_setup):
    """a peer's local failure reaches rank 0 only as a 0 in the
    MIN-reduced push-order word; rank 0 must then return an error (not CDA_OK
    with roots combined from whatever arrived).  CDA_COMM_FAULT=peer poisons
    the word before the reduce as a failed peer would."""
    from celestia_da import _lib
    c, d_ods, k = comm_setup
    os.environ["CDA_COMM_FAULT"] = "peer"
    rc, msg, word = _split_rc(c, d_ods, k)
    assert rc == _lib.CDA_ERR_DEVICE and "peer rank failed" in msg, (rc, msg)
    assert word == 0
    os.environ.pop("CDA_COMM_FAULT")
    _clean_split_matches(ctx, c, d_ods, k)


def test_abort_from_watchdog_during_agreement(ctx, comm_setup):
    """cda_comm_abort from another thread while the call waits in
    the agreement round (CDA_COMM_FAULT=stall holds it there as if a peer never
    arrived) must release the call with CDA_ERR_COMM, without touching the
    aborted communicator afterwards; a fresh communicator then works."""
    import threading
    import time

    import torch
    from celestia_da import _lib, testfactory
    c, d_ods, k = comm_setup
    _clean_split_matches(ctx, c, d_ods, k)
    k2 = 32   # a new k: the agreement round runs again
    d2 = torch.from_numpy(testfactory.random_square(k2, 11)).to(d_ods.device)
    os.environ["CDA_COMM_FAULT"] = "stall"
    out = {}

    def call():
        out["r"] = _split_rc(c, d2, k2)

    t = threading.Thread(target=call)
    t0 = time.monotonic()
    t.start()
    time.sleep(0.5)
    c.comm_abort()
    t.join(timeout=60)
    assert not t.is_alive()
    rc, msg, _ = out["r"]
    assert rc == _lib.CDA_ERR_COMM and "aborted during the call" in msg, (rc, msg)
    assert time.monotonic() - t0 < 20
    os.environ.pop("CDA_COMM_FAULT")
    c.comm_init(0, 1, _lib.comm_unique_id())
    _clean_split_matches(ctx, c, d2, k2)
