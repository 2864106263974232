#!/bin/bash
# GPU-box A/B (round 5): the current build against build_var/r05z (the build
# of the r05z evidence, before the wave-priority changes) on the default
# headline bench, interleaved.  Output: gpurun_out/<tag>/ab.txt.
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2 3 4; do
  for v in head r05z; do
    case $v in head) E="" ;; r05z) E="CDA_LIB=$PWD/celestia-app_amd/build_var/r05z/libcda.so" ;; esac
    env $E timeout -k 10 200 python -u bench.py --no-cpu --no-extras --steps 20 > "$OUT/ab_${v}_r${rep}.log" 2>&1 || exit $?
    python - "$OUT/ab_${v}_r${rep}.log" "$v" <<'PY' | tee -a "$OUT/ab.txt"
import json, sys
s = open(sys.argv[1]).read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
print(sys.argv[2], "sq/s %.1f" % j["value"], "ms/step %.3f" % j["ms_per_step"],
      {k: round(v["avg_ms"], 3) for k, v in j["stages"].items()})
PY
  done
done
