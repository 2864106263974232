#!/bin/bash
# GPU-box A/B of the latency-bound tail (round 5): the product library (the
# kRfcPad row loaded before block 0 in every RFC-6962 inner node), the same
# source built with -DCDA_RFC_ROW_LATE (the round-4 placement, 16 rounds
# ahead of use; build_var/rfclate), and the product without data-root
# schedule helpers (CDA_DR_HELPERS=0).  The whole GPU suite first, then
# interleaved bench runs:
# one k = 512 square per step and one k = 128 square per step.
# Output: gpurun_out/<tag>/ab.txt.
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/parity.log" 2>&1 || exit $?
tail -1 "$OUT/parity.log"
for rep in 1 2 3; do
  for v in new late nohelp; do
    for k in 512 128; do
      case $v in
        new) E="" ;;
        late) E="CDA_LIB=$PWD/celestia-app_amd/build_var/rfclate/libcda.so" ;;
        nohelp) E="CDA_DR_HELPERS=0" ;;
      esac
      if [ $k = 512 ]; then S="--steps 60 --warmup 40"; else S="--steps 400 --warmup 200"; fi
      env $E timeout -k 10 200 python -u bench.py --k $k --batch 1 --no-cpu --no-extras $S \
        > "$OUT/ab_${v}_k${k}_r${rep}.log" 2>&1 || exit $?
      python - "$OUT/ab_${v}_k${k}_r${rep}.log" "$v" "$k" <<'PY' | tee -a "$OUT/ab.txt"
import json, sys
s = open(sys.argv[1]).read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
st = j.get("stages", {})
print(sys.argv[2], "k", sys.argv[3], "ms/sq %.4f" % j["ms_per_step"],
      {k: round(v["avg_ms"], 4) for k, v in st.items()})
PY
    done
  done
done
