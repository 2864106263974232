#!/bin/bash
# GPU-box A/B (round 5): config 4's N = 8 shard (128 k = 128 squares per step)
# with the last NMT levels in one fused tree-top launch (CDA_TOP_FUSE = nodes
# per tree the top starts from) against the default (subtrees of 32 leaves,
# then per-level launches 8 -> 4 -> 2 -> 1).  Output: gpurun_out/<tag>/ab.txt.
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2 3; do
  for v in base tf4 tf8 tf16; do
    case $v in base) E="" ;; tf4) E="CDA_TOP_FUSE=4" ;; tf8) E="CDA_TOP_FUSE=8" ;; tf16) E="CDA_TOP_FUSE=16" ;; esac
    env $E timeout -k 10 200 python -u bench.py --batch 128 --no-cpu --no-extras --steps 20 \
      > "$OUT/ab_${v}_r${rep}.log" 2>&1 || exit $?
    python - "$OUT/ab_${v}_r${rep}.log" "$v" <<'PY' | tee -a "$OUT/ab.txt"
import json, sys
s = open(sys.argv[1]).read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
st = j.get("stages", {})
print(sys.argv[2], "sq/s %.1f" % j["value"], "ms/step %.3f" % j["ms_per_step"], "parity", j["parity"]["matched"],
      {k: round(v["avg_ms"], 3) for k, v in st.items()})
PY
  done
done
