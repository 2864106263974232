#!/bin/bash
# RS / SHA-256 spatial split sweep (run via gpurun): pipeline chunk x CU split
# (CDA_RS_CU=S:R[:G], engine.hip).  Prints one summary line per setting.
set -o pipefail
mkdir -p gpurun_out
for cfg in ${CFGS:-"0:" "32:8:1" "16:8:1" "32:16:3" "16:16:3" "32:4:1" "16:8:1:1"}; do
  chunk=${cfg%%:*}; cu=${cfg#*:}
  tag=c${chunk}_cu${cu//:/-}
  envs=""
  [ "$chunk" != 0 ] && envs="CDA_PIPELINE_CHUNK=$chunk"
  [ -n "$cu" ] && envs="$envs CDA_RS_CU=$cu"
  env $envs timeout -k 10 120 python bench.py --no-cpu --no-extras --steps 10 --warmup 2 > gpurun_out/cu_$tag.json 2> gpurun_out/cu_$tag.err || exit 1
  python - "$tag" gpurun_out/cu_$tag.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
st={k:(round(v["avg_ms"],3),v["launches"]) for k,v in d["stages"].items()}
print(sys.argv[1], round(d["value"],1), round(d["ms_per_step"],3), st, flush=True)
PY
done
