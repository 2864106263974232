#!/bin/bash
# Rehearse the N > 1 bench flows on a one-GPU box: two ranks on device 0, gloo
# for the parent group (RCCL refuses two ranks on one GPU, so the config-5
# library RCCL leg is expected to report an error, not a result).
#   (1) the driver's launcher: torch.distributed.run ... bench.py --gpus 2
#   (2) a plain `bench.py --gpus 2`: bench.py spawns its own two ranks
set -o pipefail
mkdir -p gpurun_out/n2
export CDA_BENCH_DEVICE=0 CDA_BENCH_BACKEND=gloo CDA_CONFIG5_TIMEOUT_S=90
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 1 > gpurun_out/n2/launcher.log 2> gpurun_out/n2/launcher.err \
  || exit $?
timeout -k 10 500 python bench.py --gpus 2 --steps 5 --warmup 1 > gpurun_out/n2/spawn.log 2> gpurun_out/n2/spawn.err \
  || exit $?
python - <<'PY'
import json
for f in ("launcher", "spawn"):
    s = open(f"gpurun_out/n2/{f}.log").read().strip().splitlines()
    j = json.loads([l for l in s if l.startswith('{"metric')][-1])
    print(f, j["n_gpus"], j["launch"], round(j["value"]), j["ms_per_step"], j["parity"],
          json.dumps(j["extras"].get("config5"))[:400])
PY
