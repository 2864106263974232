#!/bin/bash
# A/B of CDA_HASH_SPLIT (0: one stream; 2: the batch's two halves hashed on
# two streams) on the headline bench, alternating runs on one box.
set -e
mkdir -p gpurun_out
for rep in 1 2; do
  for v in ${SPLITS:-0 2}; do
    CDA_HASH_SPLIT=$v timeout -k 10 120 python bench.py --no-cpu --no-extras --steps 30 > gpurun_out/hsplit_$v.log 2>&1
    python - "$v" "$rep" <<'PY'
import json, sys
v, rep = sys.argv[1], sys.argv[2]
s = open(f"gpurun_out/hsplit_{v}.log").read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
print(f"rep {rep} CDA_HASH_SPLIT={v}", round(j["value"]), "sq/s", round(j["ms_per_step"], 3), "ms",
      {k: round(x["avg_ms"], 3) for k, x in j["stages"].items()}, j["parity"]["matched"], "/", j["parity"]["checked"])
PY
  done
done
