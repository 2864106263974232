"""bench.py --gpus N launcher logic, CPU only.

A plain `python bench.py --gpus N` (no torch.distributed.run) must start N
rank processes itself, from a parent that never touches the GPU; under a
launcher, WORLD_SIZE must equal --gpus or the run is refused."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_launch_mode():
    assert bench.launch_mode(1, {}) == "inprocess"
    assert bench.launch_mode(2, {}) == "spawn"
    assert bench.launch_mode(8, {}) == "spawn"
    assert bench.launch_mode(8, {"WORLD_SIZE": "8"}) == "rank"
    assert bench.launch_mode(1, {"WORLD_SIZE": "1"}) == "rank"
    assert bench.launch_mode(8, {"WORLD_SIZE": "1"}) == "mismatch"
    assert bench.launch_mode(1, {"WORLD_SIZE": "4"}) == "mismatch"
    assert bench.launch_mode(0, {}) == "mismatch"


def test_rank_commands():
    cmds = bench.rank_commands(["--gpus", "4", "--steps", "3"], 4, 29999, {"PATH": "/bin", "KEEP": "x"})
    assert len(cmds) == 4
    for g, (argv, env) in enumerate(cmds):
        assert argv[0] == sys.executable
        assert argv[-4:] == ["--gpus", "4", "--steps", "3"]
        assert os.path.basename(argv[-5]) == "bench.py"
        assert env["RANK"] == env["LOCAL_RANK"] == str(g)
        assert env["WORLD_SIZE"] == "4"
        assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29999"
        assert env["KEEP"] == "x" and env["CDA_BENCH_LAUNCHER"] == "bench.py"
        # the rank process sees a consistent launch
        assert bench.launch_mode(4, env) == "rank"


def test_free_port():
    p = bench.free_port()
    assert 0 < p < 65536


def _env(**kv):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(kv)
    return e


def test_mismatch_exits_nonzero():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"], env=_env(WORLD_SIZE="1"),
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr and r.stdout == ""


def test_spawn_propagates_rank_failure():
    # no GPU here: every spawned rank fails at torch.cuda.set_device; the
    # parent (which never imported torch) must report a failure, not 0
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--no-cpu", "--no-extras"],
                       env=_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "rank" in r.stderr and "exited with" in r.stderr
    assert r.stdout.strip() == ""


@pytest.mark.parametrize("rc,want", [(1, 1), (2, 2), (-9, 137), (-6, 134)])
def test_exit_status(rc, want):
    assert bench._exit_status(rc) == want


def _parity_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    got = bench.gather_parity({"checked": 10 + rank, "matched": 10 + rank - (rank == 1)}, world, "cpu")
    q.put((rank, got))
    dist.destroy_process_group()


def test_gather_parity_gloo():
    """Rank 0's line sums every rank's fixture checks and lists them per rank
    (world size 3 over gloo; rank 1 reports one mismatch)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = bench.free_port()
    procs = [ctx.Process(target=_parity_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(3))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = {"checked": 33, "matched": 32, "per_rank": [[10, 10], [11, 10], [12, 12]]}
    assert all(res[r] == want for r in range(3))


def test_parent_sigterm_kills_ranks(tmp_path):
    """A launcher's SIGTERM to the GPU-free parent must take the rank
    processes down with it (no orphaned ranks holding a GPU)."""
    import signal
    import time
    script = tmp_path / "fake_rank.py"
    script.write_text("import os, time\nopen(os.environ['PIDFILE'] + os.environ['RANK'], 'w').write(str(os.getpid()))\n"
                      "time.sleep(60)\n")
    code = (f"import sys; sys.path.insert(0, {ROOT!r}); import bench\n"
            f"bench.rank_commands = lambda argv, g, port, env: [([sys.executable, {str(script)!r}], "
            f"dict(env, RANK=str(r))) for r in range(g)]\n"
            f"sys.exit(bench.spawn_ranks([], 2))\n")
    env = _env(PIDFILE=str(tmp_path / "pid"))
    p = subprocess.Popen([sys.executable, "-c", code], env=env)
    pids = []
    for _ in range(100):
        time.sleep(0.1)
        files = [tmp_path / f"pid{r}" for r in range(2)]
        if all(f.exists() and f.read_text() for f in files):
            pids = [int(f.read_text()) for f in files]
            break
    assert len(pids) == 2
    p.send_signal(signal.SIGTERM)
    assert p.wait(timeout=30) == 128 + signal.SIGTERM
    time.sleep(0.5)
    for pid in pids:
        try:
            os.kill(pid, 0)
            alive = open(f"/proc/{pid}/stat").read().split()[2] != "Z"
        except (ProcessLookupError, FileNotFoundError):
            alive = False
        assert not alive, pid
