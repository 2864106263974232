#!/bin/bash
# GPU-box A/B (round 5): k = 512 batches with the RS of the next chunk on the
# context's second stream beside the hashing of the current one
# (CDA_PIPELINE_CHUNK; GF(2^16)'s RS leaves the VALU idle in its memory phases)
# and with one hash stream (CDA_HASH_SPLIT=1) against the default schedule.
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
  for v in base pc1 pc2 hs1; do
    for b in 4 16; do
      case $v in
        base) E="CDA_X=0" ;;
        pc1) E="CDA_PIPELINE_CHUNK=1" ;;
        pc2) E="CDA_PIPELINE_CHUNK=2" ;;
        hs1) E="CDA_HASH_SPLIT=1" ;;
      esac
      env $E timeout -k 10 200 python -u bench.py --k 512 --batch $b --no-cpu --no-extras --steps 10 \
        > "$OUT/ab_${v}_b${b}_r${rep}.log" 2>&1 || exit $?
      python - "$OUT/ab_${v}_b${b}_r${rep}.log" $v $b <<'PY' | tee -a "$OUT/ab.txt"
import json, sys
s = open(sys.argv[1]).read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
b = int(sys.argv[3])
print(sys.argv[2], "batch", b, "ms/sq %.4f" % (j["ms_per_step"] / b), "parity", j.get("parity"))
PY
    done
  done
done
