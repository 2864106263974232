#!/bin/bash
# GPU-box A/B (round 5): the data root's first level on lane pairs when its
# launch holds 512 threads (kPairMaxParents 256: k = 512's 256-parent first
# level), the product, against build_var/pm128 (128: a thread per parent
# there).  k = 512 GPU tests first, then interleaved benches of one / four
# k = 512 squares per step.  Output: gpurun_out/<tag>/ab.txt.
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "512 or data_root or dah" > "$OUT/parity.log" 2>&1 || exit $?
tail -1 "$OUT/parity.log"
for rep in 1 2 3; do
  for v in new pm128; do
    for b in 1 4; do
      case $v in new) E="" ;; pm128) E="CDA_LIB=$PWD/celestia-app_amd/build_var/pm128/libcda.so" ;; esac
      env $E timeout -k 10 200 python -u bench.py --k 512 --batch $b --no-cpu --no-extras --steps 30 --warmup 40 \
        > "$OUT/ab_${v}_b${b}_r${rep}.log" 2>&1 || exit $?
      python - "$OUT/ab_${v}_b${b}_r${rep}.log" "$v" "$b" <<'PY' | tee -a "$OUT/ab.txt"
import json, sys
s = open(sys.argv[1]).read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
st = j.get("stages", {})
b = int(sys.argv[3])
print(sys.argv[2], "batch", b, "ms/sq %.4f" % (j["ms_per_step"] / b), "data_root %.4f" % st["data_root"]["avg_ms"],
      "levels %.4f" % st["nmt_levels"]["avg_ms"])
PY
    done
  done
done
