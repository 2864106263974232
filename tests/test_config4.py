"""Config 4 (BASELINE.json configs[3]): a batch of independent k=128 squares
sharded across GPUs with no collective.

  * GPU: one rank's whole shard -- 128 distinct squares (indexes 0..127, the
    squares GPU 0 of an 8-GPU node processes) in ONE device submission, every
    data root and every square's row/column roots checked against the oracle
    fixture tests/golden/config4_k128.json (oracle/gen_config4.py), a sample
    of full EDSs by digest and one square byte-for-byte against the C oracle.
    Reference analogue: the block replay of app/process_proposal.go:138-152.
    Ranks 3 and 7 (squares 384.. and 896..) against config4_k128_rest.json.
  * CPU (gloo, world size 2): bench.py's rank partition and the MAX-over-ranks
    reduction of its timed region.
"""
import hashlib
import json
import os
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _fixture():
    with open(os.path.join(HERE, "golden", "config4_k128.json")) as f:
        return json.load(f)


def _sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_fixture_covers_rank0_shard():
    import bench
    g = _fixture()
    assert g["k"] == 128 and len(g["squares"]) == 128
    assert [str(i) for i in bench.shard(0, 8, 128)] == sorted(g["squares"], key=int)


def _fixture_rest():
    with open(os.path.join(HERE, "golden", "config4_k128_rest.json")) as f:
        return json.load(f)


def test_fixtures_cover_all_1024_squares():
    """config4_k128.json (rank 0, full digests) + config4_k128_rest.json
    (ranks 1..7, data roots and root digests) = every square of config 4."""
    a, b = _fixture(), _fixture_rest()
    assert b["k"] == 128 and b["first"] == 128 and b["count"] == 896
    assert sorted(map(int, a["squares"])) + sorted(map(int, b["squares"])) == list(range(1024))


@pytest.mark.gpu
@pytest.mark.parametrize("rank", [3, 7])
def test_config4_other_rank_shard_on_gpu(ctx, rank):
    """Rank g > 0's shard of the 8-GPU config (squares 128g .. 128g+127) in
    one in-place submission: every data root and every square's row/column
    roots against the oracle fixture."""
    import torch

    from celestia_da import testfactory
    import bench
    g = _fixture_rest()
    k, n = 128, 128
    W = 2 * k
    idx = list(bench.shard(rank, 8, n))
    dev = torch.device("cuda", 0)
    eds = torch.zeros(n, W * W * 512, dtype=torch.uint8, device=dev)
    for j, i in enumerate(idx):
        eds[j].view(W, W, 512)[:k, :k] = torch.from_numpy(testfactory.random_square(k, i)).to(dev).view(k, k, 512)
    rows = torch.empty(n, W * 90, dtype=torch.uint8, device=dev)
    cols = torch.empty(n, W * 90, dtype=torch.uint8, device=dev)
    roots = torch.empty(n, 32, dtype=torch.uint8, device=dev)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    ctx.extend_dah_inplace_device(k, n, eds.data_ptr(), rows.data_ptr(), cols.data_ptr(), roots.data_ptr(),
                                  status.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()
    r, c, dr = rows.cpu().numpy(), cols.cpu().numpy(), roots.cpu().numpy()
    for j, i in enumerate(idx):
        want = g["squares"][str(i)]
        assert dr[j].tobytes().hex() == want["data_root"], i
        assert _sha(r[j].reshape(W, 90)) == want["row_roots_sha256"], i
        assert _sha(c[j].reshape(W, 90)) == want["col_roots_sha256"], i


@pytest.mark.gpu
def test_config4_all_1024_squares_one_submission(ctx):
    """Config 4 as BASELINE.json configs[3] defines it at N = 1: ALL 1024
    squares in ONE in-place submission (cda_extend_dah_inplace_device) --
    a 32 GiB EDS arena, so byte offsets run far past 2^32 in every kernel.
    Submission order is rotated by 512 (position p holds square
    (p + 512) % 1024), so the squares with full EDS digests (0..127) sit at
    16-20 GiB.  Every data root and every square's row/column root digest is
    compared with the oracle fixtures, and a sample of whole EDSs by digest."""
    import torch

    import bench
    from celestia_da import testfactory
    g = _fixture()
    g["squares"].update(_fixture_rest()["squares"])
    k, n = 128, 1024
    W = 2 * k
    order = [(p + 512) % n for p in range(n)]
    dev = torch.device("cuda", 0)
    eds = torch.empty((n, W, W, 512), dtype=torch.uint8, device=dev)
    for j0, part in testfactory.random_squares(k, order):
        eds[j0:j0 + part.shape[0], :k, :k] = torch.from_numpy(part).to(dev).view(-1, k, k, 512)
    rows = torch.empty(n, W * 90, dtype=torch.uint8, device=dev)
    cols = torch.empty(n, W * 90, dtype=torch.uint8, device=dev)
    roots = torch.empty(n, 32, dtype=torch.uint8, device=dev)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    ctx.extend_dah_inplace_device(k, n, eds.data_ptr(), rows.data_ptr(), cols.data_ptr(), roots.data_ptr(),
                                  status.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()
    r, c, dr = rows.cpu().numpy(), cols.cpu().numpy(), roots.cpu().numpy()
    bad = []
    for p, i in enumerate(order):
        want = g["squares"][str(i)]
        if (dr[p].tobytes().hex() != want["data_root"] or _sha(r[p].reshape(W, 90)) != want["row_roots_sha256"]
                or _sha(c[p].reshape(W, 90)) != want["col_roots_sha256"]):
            bad.append((p, i))
    assert not bad, f"{len(bad)} squares differ from the oracle, first {bad[:4]}"
    for i in (0, 63, 127):           # at positions 512, 575, 639: offsets 16-20 GiB
        p = order.index(i)
        assert _sha(eds[p].cpu().numpy()) == g["squares"][str(i)]["eds_sha256"], (p, i)
    assert list(bench.shard(0, 1, 1024)) == list(range(1024))

    # Push-order status on this path: the same arena with
    # Q0 namespace violations in the squares at positions 700 and 1023 (the
    # one-hash-stream, 524 288-lane subtree schedule of >= 64 squares).  Only
    # those statuses are set, cda_push_order_detail_at equals a brute-force
    # first violation, and every other data root still equals the fixtures
    # (app/process_proposal.go:138-147 rejects on exactly that status).
    bad = {700: (40, 77), 1023: (127, 1)}
    want_detail = {}
    for p, (r0, c0) in bad.items():
        q0 = eds[p, :k, :k].cpu().numpy()
        q0[r0, c0, :29] = q0[0, 0, :29]
        want_detail[p] = _first_violation(q0)
        assert want_detail[p] is not None
        eds[p, r0, c0, :29] = torch.from_numpy(q0[r0, c0, :29].copy()).to(dev)
    ctx.extend_dah_inplace_device(k, n, eds.data_ptr(), rows.data_ptr(), cols.data_ptr(), roots.data_ptr(),
                                  status.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    st = status.cpu().numpy()
    assert sorted(np.nonzero(st)[0].tolist()) == sorted(bad), np.nonzero(st)[0][:8]
    assert all(st[p] == -3 for p in bad)      # CDA_ERR_PUSH_ORDER
    for p in bad:
        assert ctx.push_order_detail_at(p) == want_detail[p], p
    assert ctx.push_order_detail_at(0) == (-1, 0, 0)
    dr = roots.cpu().numpy()
    diff = [p for p, i in enumerate(order) if p not in bad and dr[p].tobytes().hex() != g["squares"][str(i)]["data_root"]]
    assert not diff, f"{len(diff)} ordered squares changed their data root, first {diff[:4]}"
    with pytest.raises(Exception):
        ctx.push_order_detail_at(n)            # beyond the last device batch


def _first_violation(q0):
    """Brute-force nmt push-order check of one Q0 (k x k x 512): the smallest
    (axis, index, position) whose namespace is below its predecessor's (rows
    before columns), as cda_push_order_detail reports."""
    k = q0.shape[0]
    ns = [[bytes(q0[r, c, :29]) for c in range(k)] for r in range(k)]
    bad = [(0, r, c) for r in range(k) for c in range(1, k) if ns[r][c] < ns[r][c - 1]]
    bad += [(1, c, r) for c in range(k) for r in range(1, k) if ns[r][c] < ns[r - 1][c]]
    return min(bad) if bad else None


@pytest.mark.gpu
def test_push_order_status_k512_batch_of_two(ctx):
    """Config 3's GF(2^16) path with a Q0 namespace violation in the second
    square of a batch of 2 (in place): status [0, CDA_ERR_PUSH_ORDER], the
    detail of square 1 equals a brute-force first violation, and square 0's
    data root equals tests/golden/k512.json."""
    import torch

    from celestia_da import testfactory
    with open(os.path.join(HERE, "golden", "k512.json")) as f:
        g = json.load(f)["squares"]
    k, n = 512, 2
    W = 2 * k
    dev = torch.device("cuda", 0)
    q0 = testfactory.random_square(k, 0).reshape(k, k, 512)
    bad = q0.copy()
    bad[300, 5, :29] = bad[0, 0, :29]
    bad[2, 400, :29] = bad[0, 0, :29]
    want = _first_violation(bad)
    assert want is not None
    eds = torch.empty((n, W, W, 512), dtype=torch.uint8, device=dev)
    eds[0, :k, :k] = torch.from_numpy(q0).to(dev)
    eds[1, :k, :k] = torch.from_numpy(bad).to(dev)
    rows = torch.empty(n, W * 90, dtype=torch.uint8, device=dev)
    cols = torch.empty(n, W * 90, dtype=torch.uint8, device=dev)
    roots = torch.empty(n, 32, dtype=torch.uint8, device=dev)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    ctx.extend_dah_inplace_device(k, n, eds.data_ptr(), rows.data_ptr(), cols.data_ptr(), roots.data_ptr(),
                                  status.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    assert status.cpu().tolist() == [0, -3]
    assert ctx.push_order_detail_at(1) == want
    assert ctx.push_order_detail_at(0) == (-1, 0, 0)
    assert roots[0].cpu().numpy().tobytes().hex() == g["0"]["data_root"]
    del eds
    torch.cuda.empty_cache()


@pytest.mark.gpu
@pytest.mark.parametrize("world,rank", [(2, 1), (4, 2)])
def test_config4_multi_gpu_shard_one_submission(ctx, world, rank):
    """The per-GPU shard of config 4 at N = 2 and N = 4 (BASELINE.json
    configs[3]: 1024 squares split over N GPUs): rank g's 1024 / N squares in
    ONE in-place submission, exactly what bench.py's rank g submits (16 and 8
    GiB arenas: offsets past 2^32 at N = 2), every data root and root digest
    against the oracle fixtures."""
    import torch

    import bench
    from celestia_da import testfactory
    g = _fixture()
    g["squares"].update(_fixture_rest()["squares"])
    k = 128
    n = 1024 // world
    W = 2 * k
    idx = list(bench.shard(rank, world, n))
    dev = torch.device("cuda", 0)
    eds = torch.empty((n, W, W, 512), dtype=torch.uint8, device=dev)
    for j0, part in testfactory.random_squares(k, idx):
        eds[j0:j0 + part.shape[0], :k, :k] = torch.from_numpy(part).to(dev).view(-1, k, k, 512)
    rows = torch.empty(n, W * 90, dtype=torch.uint8, device=dev)
    cols = torch.empty(n, W * 90, dtype=torch.uint8, device=dev)
    roots = torch.empty(n, 32, dtype=torch.uint8, device=dev)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    ctx.extend_dah_inplace_device(k, n, eds.data_ptr(), rows.data_ptr(), cols.data_ptr(), roots.data_ptr(),
                                  status.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()
    r, c, dr = rows.cpu().numpy(), cols.cpu().numpy(), roots.cpu().numpy()
    bad = [(p, i) for p, i in enumerate(idx)
           if dr[p].tobytes().hex() != g["squares"][str(i)]["data_root"]
           or _sha(r[p].reshape(W, 90)) != g["squares"][str(i)]["row_roots_sha256"]
           or _sha(c[p].reshape(W, 90)) != g["squares"][str(i)]["col_roots_sha256"]]
    assert not bad, f"{len(bad)} squares differ from the oracle, first {bad[:4]}"
    del eds
    torch.cuda.empty_cache()


def test_shard_partitions_config4():
    import bench
    for world in (1, 2, 4, 8):
        per = 1024 // world
        seen = [i for r in range(world) for i in bench.shard(r, world, per)]
        assert seen == list(range(1024))


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["inplace", "packed"])
def test_config4_rank_shard_on_gpu(ctx, layout):
    import torch

    import coracle
    from celestia_da import testfactory
    g = _fixture()
    k, n = 128, 128
    W = 2 * k
    dev = torch.device("cuda", 0)
    ods = np.stack([testfactory.random_square(k, i) for i in range(n)])
    d_ods = torch.from_numpy(ods).to(dev)
    eds = torch.zeros(n, W * W * 512, dtype=torch.uint8, device=dev)
    rows = torch.empty(n, W * 90, dtype=torch.uint8, device=dev)
    cols = torch.empty(n, W * 90, dtype=torch.uint8, device=dev)
    roots = torch.empty(n, 32, dtype=torch.uint8, device=dev)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    if layout == "inplace":
        eds.view(n, W, W, 512)[:, :k, :k] = d_ods.view(n, k, k, 512)
        ctx.extend_dah_inplace_device(k, n, eds.data_ptr(), rows.data_ptr(), cols.data_ptr(), roots.data_ptr(),
                                      status.data_ptr(), stream)
    else:
        ctx.extend_dah_device(d_ods.data_ptr(), k, n, eds.data_ptr(), rows.data_ptr(), cols.data_ptr(),
                              roots.data_ptr(), status.data_ptr(), stream)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()
    r, c, dr = rows.cpu().numpy(), cols.cpu().numpy(), roots.cpu().numpy()
    for i in range(n):
        want = g["squares"][str(i)]
        assert _sha(ods[i]) == want["ods_sha256"], i
        assert dr[i].tobytes().hex() == want["data_root"], i
        assert _sha(r[i].reshape(W, 90)) == want["row_roots_sha256"], i
        assert _sha(c[i].reshape(W, 90)) == want["col_roots_sha256"], i
    for i in (0, 1, 63, 64, 126, 127):
        assert _sha(eds[i].cpu().numpy()) == g["squares"][str(i)]["eds_sha256"], i
    e_eds, e_rows, e_cols, e_root = coracle.cpu_baseline(ods[77], 8)
    assert np.array_equal(eds[77].cpu().numpy().reshape(-1, 512), e_eds)
    assert np.array_equal(r[77].reshape(W, 90), e_rows) and np.array_equal(c[77].reshape(W, 90), e_cols)
    assert dr[77].tobytes() == e_root


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench_worker(rank, world, port, q):
    import time

    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def reduce_max(x):
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    steps, dt = 4, 0.05 * (rank + 1)          # rank 1 is the slow one
    el = bench.time_region(lambda: time.sleep(dt), steps, lambda: None, world, reduce_max, dist.barrier)
    q.put((rank, el, list(bench.shard(rank, world, 1024 // world))))
    dist.destroy_process_group()


def test_bench_rank_partition_and_max_time_gloo():
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    msgs = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, el0, s0), (_, el1, s1) = msgs
    assert el0 == el1, "every rank must report the same (max) time"
    assert el0 >= 4 * 0.1 - 1e-3, "the max over ranks is the slow rank's time"
    assert s0 == list(range(512)) and s1 == list(range(512, 1024))


def test_stage_report_is_per_step():
    """A stage marked several times per step (the levels: wide launches, then
    the tree top) is reported per step when `steps` is given, and its rate
    counts the whole stage's compressions once per step."""
    sys.path.insert(0, ROOT)
    import bench
    st = {"nmt_levels": (2.0, 4), "nmt_leaves": (3.0, 2)}     # 2 steps: levels marked twice per step
    r = bench.stage_report(st, 512, 1, False, 2)
    assert r["nmt_levels"]["avg_ms"] == 1.0 and r["nmt_leaves"]["avg_ms"] == 1.5
    want = bench.compressions(512)["nmt_levels"] / 1e-3
    assert abs(r["nmt_levels"]["compressions_per_s"] - want) < 1e-6 * want


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 7, 63, 64, 65])
def test_inplace_batch_sizes_around_schedule_switches(ctx, n):
    """Batch sizes on both sides of the engine's schedule switches -- one
    codeword per RS workgroup below two per CU (a single square), the XCD-slice
    Q0 launch, the two-stream hash split below 64 squares and one stream from
    64 -- each against the oracle fixture (squares 0..n-1)."""
    import torch

    from celestia_da import testfactory
    g = _fixture()["squares"]
    k = 128
    W = 2 * k
    dev = torch.device("cuda", 0)
    eds = torch.empty((n, W, W, 512), dtype=torch.uint8, device=dev)
    for j0, part in testfactory.random_squares(k, list(range(n))):
        eds[j0:j0 + part.shape[0], :k, :k] = torch.from_numpy(part).to(dev).view(-1, k, k, 512)
    rows = torch.empty(n, W * 90, dtype=torch.uint8, device=dev)
    cols = torch.empty(n, W * 90, dtype=torch.uint8, device=dev)
    roots = torch.empty(n, 32, dtype=torch.uint8, device=dev)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    ctx.extend_dah_inplace_device(k, n, eds.data_ptr(), rows.data_ptr(), cols.data_ptr(), roots.data_ptr(),
                                  status.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()
    r, c, dr = rows.cpu().numpy(), cols.cpu().numpy(), roots.cpu().numpy()
    for i in range(n):
        assert dr[i].tobytes().hex() == g[str(i)]["data_root"], i
        assert _sha(r[i].reshape(W, 90)) == g[str(i)]["row_roots_sha256"], i
        assert _sha(c[i].reshape(W, 90)) == g[str(i)]["col_roots_sha256"], i
    for i in {0, n - 1}:
        if "eds_sha256" in g[str(i)]:
            assert _sha(eds[i].cpu().numpy()) == g[str(i)]["eds_sha256"], i
