#!/bin/bash
# GPU side of tools/rs16_phase_probe.sh: k = 512 bench passes (4 squares per
# step) per library variant; stage times only.
set -e
mkdir -p gpurun_out
for v in base rs16_probe1 rs16_probe2; do
  if [ $v = base ]; then L=celestia-app_amd/libcda.so; else L=tools/var/$v/libcda.so; fi
  CDA_LIB=$PWD/$L CDA_BENCH_NOCHECK=1 timeout -k 10 150 python bench.py --k 512 --batch 4 --no-cpu --no-extras \
    --steps 10 > gpurun_out/phase16_$v.log 2>&1
  python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
s = open(f"gpurun_out/phase16_{v}.log").read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
print(v, round(j["value"], 1), "sq/s", {k: round(x["avg_ms"], 3) for k, x in j["stages"].items()})
PY
done
