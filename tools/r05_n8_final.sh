#!/bin/bash
# GPU-box check (end of round 5): one GPU's rate on config 4's N = 8 shard
# (128 squares per step) and N = 4 / N = 2 shards (256 / 512) against the full
# 1 024-square batch, interleaved on one box, with the final build's defaults.
# Output: gpurun_out/<tag>/ab.txt.
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2 3; do
  for B in 1024 128 256 512; do
    timeout -k 10 200 python -u bench.py --batch $B --no-cpu --no-extras --steps 20 \
      > "$OUT/n_b${B}_r${rep}.log" 2>&1 || exit $?
    python - "$OUT/n_b${B}_r${rep}.log" $B <<'PY' | tee -a "$OUT/ab.txt"
import json, sys
s = open(sys.argv[1]).read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
print("batch", sys.argv[2], "sq/s %.1f" % j["value"], "ms/step %.3f" % j["ms_per_step"], "parity", j.get("parity", {}).get("matched"))
PY
  done
done
