#!/bin/bash
# Rehearse the N > 1 bench flows on a one-GPU box: N ranks on device 0, gloo
# for the parent group (RCCL refuses several ranks on one GPU, so the config-5
# library RCCL leg is expected to report an error, not a result).  Each rank
# and its config-5 child use the GPU: keep 2 N <= 16 (the box's GPU-process cap).
#   (1) the driver's launcher: torch.distributed.run ... bench.py --gpus N
#   (2) a plain `bench.py --gpus N`: bench.py spawns its own N ranks
# Usage: bash tools/rehearse_n.sh N
set -o pipefail
N=${1:?N}
OUT=gpurun_out/n$N
mkdir -p $OUT
export CDA_BENCH_DEVICE=0 CDA_BENCH_BACKEND=gloo CDA_CONFIG5_TIMEOUT_S=150
timeout -k 10 560 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus $N --steps 3 --warmup 1 > $OUT/launcher.log 2> $OUT/launcher.err \
  || exit $?
timeout -k 10 560 python bench.py --gpus $N --steps 3 --warmup 1 > $OUT/spawn.log 2> $OUT/spawn.err \
  || exit $?
python - "$OUT" <<'PY'
import json, sys
out = sys.argv[1]
for f in ("launcher", "spawn"):
    s = open(f"{out}/{f}.log").read().strip().splitlines()
    j = json.loads([l for l in s if l.startswith('{"metric')][-1])
    print(f, j["n_gpus"], j["launch"], round(j["value"]), j["ms_per_step"], j["parity"],
          json.dumps(j["extras"].get("config5"))[:400])
PY
