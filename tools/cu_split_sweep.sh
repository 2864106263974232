#!/bin/bash
# CU-partitioned batch pipeline (CDA_RS_CUS = CUs for the RS stream, the
# hashing on the rest; CDA_PIPELINE_CHUNK = squares per chunk) on the headline
# bench.  One line per setting: squares/s, ms per step, parity.
set -o pipefail
mkdir -p gpurun_out/cusplit
for c in ${CHUNKS:-16 32}; do for cus in ${CUS_LIST:-0 24 32 48}; do
  tag=c${c}_cus${cus}
  CDA_RS_CUS=$cus CDA_PIPELINE_CHUNK=$c timeout -k 10 120 python bench.py --no-cpu --no-extras --steps ${STEPS:-20} \
    > gpurun_out/cusplit/$tag.log 2>&1 || { tail -5 gpurun_out/cusplit/$tag.log; exit 1; }
  python - "$tag" <<'PY'
import json, sys
t = sys.argv[1]
s = open(f"gpurun_out/cusplit/{t}.log").read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
print(t, round(j["value"]), "sq/s", round(j["ms_per_step"], 3), "ms", "parity", j["parity"]["matched"], "/", j["parity"]["checked"], flush=True)
PY
done; done
timeout -k 10 120 python bench.py --no-cpu --no-extras --steps ${STEPS:-20} > gpurun_out/cusplit/serial.log 2>&1 && python - <<'PY'
import json
s = open("gpurun_out/cusplit/serial.log").read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
print("serial default", round(j["value"]), "sq/s", round(j["ms_per_step"], 3), "ms")
PY
