#!/bin/bash
# RS/SHA co-residency sweep (run via gpurun): library variant x pipeline chunk x
# RS stream priority.  Prints one summary line per setting.
set -o pipefail
mkdir -p gpurun_out
for so in ${VARIANTS:-base rs192}; do
  for cfg in ${CFGS:-"0:" "64:" "32:" "64:-1" "32:-1" "16:-1"}; do
    chunk=${cfg%%:*}; prio=${cfg#*:}
    tag=${so}_c${chunk}_p${prio}
    envs="CDA_LIB=$PWD/celestia-app_amd/variants/libcda_$so.so"
    [ "$chunk" != 0 ] && envs="$envs CDA_PIPELINE_CHUNK=$chunk"
    [ -n "$prio" ] && envs="$envs CDA_RS_PRIORITY=$prio"
    env $envs timeout -k 10 120 python bench.py --no-cpu --no-extras --steps 10 --warmup 2 > gpurun_out/ov_$tag.json 2> gpurun_out/ov_$tag.err || exit 1
    python - "$tag" gpurun_out/ov_$tag.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
st={k:(round(v["avg_ms"],3),v["launches"]) for k,v in d["stages"].items()}
print(sys.argv[1], round(d["value"],1), round(d["ms_per_step"],3), st, flush=True)
PY
  done
done
