#!/bin/bash
# GPU-box A/B (round 5): the new hash schedule for k = 128 batches (one stream
# from 64 squares up, subtree launches targeting 524288 lanes) against the
# round-4 rule (two streams up to 256 squares, 131072 lanes; emulated with
# CDA_HASH_SPLIT / CDA_SUBTREE_LANES) at every shard size config 4 reaches
# (1024 / N squares per GPU for N = 1, 2, 4, 8, 16) and two smaller batches.
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
  for b in 1024 512 256 128 64 32 16; do
    for v in old new; do
      if [ $v = old ]; then
        HS=1; [ $b -le 256 ] && HS=2
        E="CDA_SUBTREE_LANES=131072 CDA_HASH_SPLIT=$HS"
      else
        E="CDA_X=0"
      fi
      env $E timeout -k 10 200 python -u bench.py --batch $b --no-cpu --no-extras --steps 20 > "$OUT/${v}_b${b}_r${rep}.log" 2>&1 || exit $?
      python - "$OUT/${v}_b${b}_r${rep}.log" $v $b <<'PY' | tee -a "$OUT/ab.txt"
import json, sys
s = open(sys.argv[1]).read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
st = j.get("stages", {})
print(sys.argv[2], "batch", sys.argv[3], "sq/s %.1f" % j["value"], "ms/step %.3f" % j["ms_per_step"],
      "parity", j.get("parity", {}).get("matched"), {k: round(v["avg_ms"], 3) for k, v in st.items()})
PY
    done
  done
done
