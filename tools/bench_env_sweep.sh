#!/bin/bash
# Bench the default libcda.so under several environment settings (run via gpurun).
# Usage: tools/bench_env_sweep.sh VAR "v1 v2 ..." [bench args]
set -o pipefail
mkdir -p gpurun_out
VAR=$1; VALS=$2; shift 2
for v in $VALS; do
  env $VAR=$v timeout -k 10 120 python bench.py --no-cpu --no-extras --steps 10 --warmup 2 "$@" > gpurun_out/env_$v.json 2> gpurun_out/env_$v.err || exit 1
  python - "$VAR=$v" gpurun_out/env_$v.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
st={k:(round(v["avg_ms"],3),v["launches"]) for k,v in d["stages"].items()}
print(sys.argv[1], round(d["value"],1), round(d["ms_per_step"],3), st)
PY
done
