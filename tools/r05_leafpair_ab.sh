#!/bin/bash
# GPU-box A/B of the lane-pair leaf kernel (round 5): product (leaf launches of
# <= 65 536 cells on lane pairs) against CDA_LEAF_PAIR_MAX=0 (one lane per
# cell everywhere).  The whole GPU suite first, then interleaved benches of
# one / two k = 128 squares per step and one k = 64 square, and bench.py's
# own single-square latency figure (extras, --latency-only style run).
# Output: gpurun_out/<tag>/ab.txt.
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/parity.log" 2>&1 || exit $?
tail -1 "$OUT/parity.log"
for rep in 1 2 3; do
  for v in pair single; do
    for cfg in "128 1" "128 2" "64 1"; do
      set -- $cfg
      case $v in pair) E="" ;; single) E="CDA_LEAF_PAIR_MAX=0" ;; esac
      env $E timeout -k 10 200 python -u bench.py --k $1 --batch $2 --no-cpu --no-extras --steps 400 --warmup 200 \
        > "$OUT/ab_${v}_k$1_b$2_r${rep}.log" 2>&1 || exit $?
      python - "$OUT/ab_${v}_k$1_b$2_r${rep}.log" "$v" "$1" "$2" <<'PY' | tee -a "$OUT/ab.txt"
import json, sys
s = open(sys.argv[1]).read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
st = j.get("stages", {})
print(sys.argv[2], "k", sys.argv[3], "batch", sys.argv[4], "ms/step %.4f" % j["ms_per_step"],
      {k: round(v["avg_ms"], 4) for k, v in st.items()})
PY
    done
  done
done
