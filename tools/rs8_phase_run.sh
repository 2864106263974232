#!/bin/bash
# GPU side of tools/rs8_phase_probe.sh: one bench pass per library variant,
# stage times only (outputs of the probe variants are wrong by construction).
set -e
mkdir -p gpurun_out
for v in base probe1 probe2 probe3; do
  if [ $v = base ]; then L=celestia-app_amd/libcda.so; else L=tools/var/$v/libcda.so; fi
  CDA_LIB=$PWD/$L CDA_BENCH_NOCHECK=1 timeout -k 10 120 python bench.py --no-cpu --no-extras --steps 10 \
    > gpurun_out/phase_$v.log 2>&1
  python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
s = open(f"gpurun_out/phase_{v}.log").read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
print(v, round(j["value"]), {k: x["avg_ms"] for k, x in j["stages"].items()})
PY
done
