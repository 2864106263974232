#!/bin/bash
# A/B of the k = 128 bitsliced RS kernels (CDA_RS8_BS=1: 4 codewords per
# workgroup, 2: half-footprint) on the headline bench; stage times per variant.
set -e
mkdir -p gpurun_out
for v in ${VARIANTS:-1 2}; do
  CDA_RS8_BS=$v timeout -k 10 120 python bench.py --no-cpu --no-extras --steps ${STEPS:-20} > gpurun_out/rs8_ab_$v.log 2>&1
  python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
s = open(f"gpurun_out/rs8_ab_{v}.log").read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
print("CDA_RS8_BS=" + v, round(j["value"]), "sq/s", {k: round(x["avg_ms"], 3) for k, x in j["stages"].items()})
PY
done
