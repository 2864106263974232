"""Multi-process tests of the config-5 orchestration (celestia_da.dist) over
gloo on CPU, world sizes 1, 2 and 4: the row-block / all-to-all / column-block
/ gather / combine data movement must reproduce the single-square oracle."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, k, port, q, swap):
    import sys
    for p in (HERE, os.path.join(os.path.dirname(HERE), "celestia-app_amd"), os.path.join(os.path.dirname(HERE), "oracle")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    import coracle
    from celestia_da import dist as cdist
    from split_cpu_ops import CpuSplitOps

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ods = coracle.random_square(k, 5).reshape(k, k, 512).copy()
    if swap:
        ods[1, 2, :29], ods[1, 3, :29] = ods[1, 3, :29].copy(), ods[1, 2, :29].copy()
    R = k // world
    mine = torch.from_numpy(ods[rank * R:(rank + 1) * R].copy())
    rb, block, res = cdist.extend_dah_split(mine, k, CpuSplitOps(), rank, world)
    if rank == 0:
        rows, cols, root, err = res
        q.put(("root", root.numpy().tobytes(), int(err.item()), rows.numpy().copy(), cols.numpy().copy()))
    q.put(("block", rank, block.numpy().copy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 4])
def test_split_square_matches_oracle(world):
    import coracle
    k = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, k, port, q, False)) for r in range(world)]
    for p in procs:
        p.start()
    msgs = [q.get(timeout=120) for _ in range(world + 1)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ods = coracle.random_square(k, 5)
    eds, rows, cols, root = coracle.extend_dah(ods)
    eds = eds.reshape(2 * k, 2 * k, 512)
    C = 2 * k // world
    for m in msgs:
        if m[0] == "root":
            assert m[1] == root
            assert m[2] == 0xFFFFFFFF
            assert np.array_equal(m[3], rows) and np.array_equal(m[4], cols)
        else:
            _, rank, block = m
            assert np.array_equal(block, eds[:, rank * C:(rank + 1) * C])


def test_split_push_order_error_reduced_across_ranks():
    k, world = 8, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, k, port, q, True)) for r in range(world)]
    for p in procs:
        p.start()
    msgs = [q.get(timeout=120) for _ in range(world + 1)]
    for p in procs:
        p.join(timeout=60)
    err = [m for m in msgs if m[0] == "root"][0][2]
    assert err == (0 << 24) | (1 << 12) | 3      # row 1, push position 3


def _failing_worker(rank, world, k, port, q):
    import sys
    for p in (HERE, os.path.join(os.path.dirname(HERE), "celestia-app_amd"), os.path.join(os.path.dirname(HERE), "oracle")):
        sys.path.insert(0, p)
    import torch.distributed as dist

    import coracle
    from celestia_da import dist as cdist
    from split_cpu_ops import CpuSplitOps

    class Flaky(CpuSplitOps):
        def cols(self, block, k, col0, err):
            if rank == 1:
                raise RuntimeError("injected column-step failure")
            return super().cols(block, k, col0, err)

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ods = coracle.random_square(k, 5).reshape(k, k, 512)
    R = k // world
    errors = []
    mine = torch.from_numpy(ods[rank * R:(rank + 1) * R].copy())
    cdist.extend_dah_split(mine, k, Flaky(), rank, world, on_error=errors.append)
    flag = torch.tensor([len(errors)])
    dist.all_reduce(flag)                      # every rank reaches the same collectives
    q.put((rank, [str(e) for e in errors], int(flag.item())))
    dist.destroy_process_group()


def test_split_local_failure_does_not_deadlock():
    """bench.py's config-5 run passes on_error: a local failure on one rank
    must not leave the other ranks blocked in the all-to-all / gathers."""
    k, world = 8, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_failing_worker, args=(r, world, k, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    msgs = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert msgs[0][1] == [] and msgs[1][1] == ["injected column-step failure"]
    assert all(m[2] == 1 for m in msgs)
