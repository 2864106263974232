#!/bin/bash
# GPU-box A/B (round 5): one GPU's rate on config 4's N = 8 shard (128 squares
# per step) against the full 1 024-square batch on the same box, with the
# schedule knobs that change the small shape: one hash stream
# (CDA_HASH_SPLIT=1), subtree lane target 262 144 (4 waves per SIMD of 64-leaf
# subtrees), and the RS chunk pipeline (CDA_PIPELINE_CHUNK=32).
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2; do
  for v in b1024 base hs1 sl256k pc32; do
    B=128; E="CDA_X=0"
    case $v in
      b1024) B=1024 ;;
      hs1) E="CDA_HASH_SPLIT=1" ;;
      sl256k) E="CDA_SUBTREE_LANES=262144" ;;
      pc32) E="CDA_PIPELINE_CHUNK=32" ;;
    esac
    env $E timeout -k 10 200 python -u bench.py --batch $B --no-cpu --no-extras --steps 20 \
      > "$OUT/n8_${v}_r${rep}.log" 2>&1 || exit $?
    python - "$OUT/n8_${v}_r${rep}.log" $v <<'PY' | tee -a "$OUT/ab.txt"
import json, sys
s = open(sys.argv[1]).read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
st = j.get("stages", {})
print(sys.argv[2], "sq/s %.1f" % j["value"], "ms/step %.3f" % j["ms_per_step"], "parity", j.get("parity", {}).get("matched"),
      {k: round(v["avg_ms"], 3) for k, v in st.items()})
PY
  done
done
