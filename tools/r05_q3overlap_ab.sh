#!/bin/bash
# GPU-box A/B of CDA_LEAF_Q3_OVERLAP (round 5): the leaves of Q0 | Q1 and Q2
# on a lowest-priority stream beside the RS Q3 launch (batches up to 4
# squares) against the serial schedule.  Its GPU test and the pipeline / push-
# order tests first, then interleaved benches: one / two k = 128 squares and
# one / two k = 512 squares per step.  Output: gpurun_out/<tag>/ab.txt.
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "q3_overlap or pipeline or push_order or fault" > "$OUT/parity.log" 2>&1 || exit $?
tail -1 "$OUT/parity.log"
for rep in 1 2 3; do
  for v in serial overlap; do
    for cfg in "128 1" "128 2" "512 1" "512 2"; do
      set -- $cfg
      case $v in serial) E="" ;; overlap) E="CDA_LEAF_Q3_OVERLAP=4" ;; esac
      if [ $1 = 512 ]; then S="--steps 30 --warmup 40"; else S="--steps 400 --warmup 200"; fi
      env $E timeout -k 10 200 python -u bench.py --k $1 --batch $2 --no-cpu --no-extras $S \
        > "$OUT/ab_${v}_k$1_b$2_r${rep}.log" 2>&1 || exit $?
      python - "$OUT/ab_${v}_k$1_b$2_r${rep}.log" "$v" "$1" "$2" <<'PY' | tee -a "$OUT/ab.txt"
import json, sys
s = open(sys.argv[1]).read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
print(sys.argv[2], "k", sys.argv[3], "batch", sys.argv[4], "ms/step %.4f" % j["ms_per_step"])
PY
    done
  done
done
