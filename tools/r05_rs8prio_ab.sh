#!/bin/bash
# GPU-box A/B (round 5): the GF(2^8) bitsliced encoder with s_setprio around
# its load and store phases (CDA_RS8_PRIO=1) against the same build without
# (CDA_RS8_PRIO=0, the flag read but not set) and the build before the flag
# (build_var/old8).  The GPU suite with CDA_RS8_PRIO=1 first, then
# interleaved benches: config 4 (1 024 squares), 128 squares, one square.
# Output: gpurun_out/<tag>/ab.txt.
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
CDA_RS8_PRIO=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/parity.log" 2>&1 || exit $?
tail -1 "$OUT/parity.log"
for rep in 1 2 3; do
  for v in old new0 new1; do
    for b in 1024 128 1; do
      case $v in
        old) E="CDA_LIB=$PWD/celestia-app_amd/build_var/old8/libcda.so" ;;
        new0) E="CDA_RS8_PRIO=0" ;;
        new1) E="CDA_RS8_PRIO=1" ;;
      esac
      if [ $b = 1 ]; then S="--steps 400 --warmup 200"; else S="--steps 10 --warmup 3"; fi
      env $E timeout -k 10 200 python -u bench.py --batch $b --no-cpu --no-extras $S \
        > "$OUT/ab_${v}_b${b}_r${rep}.log" 2>&1 || exit $?
      python - "$OUT/ab_${v}_b${b}_r${rep}.log" "$v" "$b" <<'PY' | tee -a "$OUT/ab.txt"
import json, sys
s = open(sys.argv[1]).read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
st = j.get("stages", {})
print(sys.argv[2], "batch", sys.argv[3], "sq/s %.1f" % j["value"], "ms/step %.4f" % j["ms_per_step"],
      "RS %.4f" % sum(st[x]["avg_ms"] for x in ("rs_q0", "rs_q3") if x in st))
PY
    done
  done
done
