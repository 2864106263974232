"""Block-replay throughput (celestia_da.replay): ProcessProposal's DA check
over many blocks, txs on the host -> data roots (app/process_proposal.go:122-152).

Times three forms over the same seeded full blocks (blobfactory.full_block):
  * replay     -- host layout per block, squares written on the GPU into one
                  batch per size, one cda_extend_dah_device per batch;
  * per_block  -- cda_construct_extend_dah once per block (host txs in, roots
                  out; the single-block ProcessProposal call);
  * plan       -- the host layout alone (the part neither form moves to the GPU).
Every replay data root is checked against the per-block call's before timing.
Host tx bytes cross PCIe in both forms: these are end-to-end, PCIe-inclusive
rates, not the bench's HBM-resident headline.

  python tools/replay_bench.py --blocks 64 --k 128 --reps 5
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=64)
    ap.add_argument("--k", type=int, default=128)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    from celestia_da import blobfactory, default_context, replay, square
    ctx = default_context()
    blocks = [blobfactory.full_block(1000 + s, a.k) for s in range(a.blocks)]
    sizes = replay.plan(blocks, a.k)[0]
    print(f"[replay_bench] {a.blocks} blocks, sizes {sorted(set(sizes))}, "
          f"{sum(sum(len(t) for t in b) for b in blocks) / 2**20:.1f} MiB of txs", flush=True)

    res = replay.replay(blocks, max_square_size=a.k, ctx=ctx)
    want = [square.construct_extend_dah(b, a.k, ctx=ctx)[4] for b in blocks]
    bad = sum(r.data_root != w for r, w in zip(res, want))
    assert bad == 0, f"{bad} data roots differ from the per-block path"

    def timed(fn):
        ts = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
        return sorted(ts)[len(ts) // 2]

    t_replay = timed(lambda: replay.replay(blocks, max_square_size=a.k, ctx=ctx))
    t_block = timed(lambda: [square.construct_extend_dah(b, a.k, ctx=ctx) for b in blocks])
    t_plan = timed(lambda: replay.plan(blocks, a.k))
    out = {"blocks": a.blocks, "k": a.k, "reps": a.reps, "parity": f"{a.blocks - bad}/{a.blocks}",
           "replay_blocks_per_s": a.blocks / t_replay, "replay_ms_per_block": 1e3 * t_replay / a.blocks,
           "per_block_blocks_per_s": a.blocks / t_block, "per_block_ms_per_block": 1e3 * t_block / a.blocks,
           "plan_ms_per_block": 1e3 * t_plan / a.blocks}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
