#!/bin/bash
# Batch-pipeline sweep: CDA_PIPELINE_CHUNK (squares per chunk, 0 = serial) x
# CDA_RS8_LDS (LDS per RS workgroup; 98304 = one RS workgroup per CU) on the
# headline bench.  One line per setting: squares/s and per-step stage ms.
set -e
mkdir -p gpurun_out
for hw in ${HASH_WG_LIST:-0}; do for lds in ${LDS_LIST:-0 98304}; do
  for c in ${CHUNKS:-0 64 32 16}; do
    tag=c${c}_lds${lds}_hw${hw}
    CDA_HASH_WG_PER_CU=$hw CDA_PIPELINE_CHUNK=$c CDA_RS8_LDS=$lds timeout -k 10 120 python bench.py --no-cpu --no-extras --steps ${STEPS:-20} \
      > gpurun_out/pipe_$tag.log 2>&1
    python - "$tag" <<'PY'
import json, sys
t = sys.argv[1]
s = open(f"gpurun_out/pipe_{t}.log").read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
print(t, round(j["value"]), "sq/s", round(j["ms_per_step"], 3), "ms",
      {k: round(x["avg_ms"], 3) for k, x in j["stages"].items()}, "parity", j.get("parity"))
PY
  done
done
done
