#!/bin/bash
# Rehearse the driver's N > 1 bench flow on a one-GPU box: two ranks on device
# 0, gloo for the parent group (RCCL refuses two ranks on one GPU, so the
# config-5 library RCCL leg is expected to report an error, not a result).
set -o pipefail
mkdir -p gpurun_out/n2
CDA_BENCH_DEVICE=0 CDA_BENCH_BACKEND=gloo CDA_CONFIG5_TIMEOUT_S=90 timeout -k 10 500 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
  bench.py --gpus 2 --steps 5 --warmup 1 > gpurun_out/n2/bench.log 2> gpurun_out/n2/bench.err
rc=$?
echo rc=$rc
grep -c '"metric"' gpurun_out/n2/bench.log
python - <<'PY'
import json
s = open("gpurun_out/n2/bench.log").read().strip().splitlines()
j = json.loads([l for l in s if l.startswith('{"metric')][-1])
print(j["n_gpus"], round(j["value"]), j["ms_per_step"], j["parity"], json.dumps(j["extras"].get("config5"))[:600])
PY
