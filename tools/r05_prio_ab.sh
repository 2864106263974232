#!/bin/bash
# GPU-box A/B (round 5): the GF(2^16) encoder with s_setprio around its load
# and store phases (2 while loading, 0 in the butterflies and exchanges, 1 in
# the LOW FFT / store phase).  r05ab: a -DCDA_BS16_SETPRIO build for every
# launch (build_var/prio) against the product of then; since: RsJob::prio,
# set for launches of <= CDA_RS16_PRIO_MAX squares (default 4), against
# CDA_RS16_PRIO_MAX=0.  GF(2^16) GPU tests first, then interleaved benches at
# k = 512 batch 1 / 2 / 4 / 16.  Output: gpurun_out/<tag>/.
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "512 or gf16 or codec or linear" > "$OUT/parity.log" 2>&1 || exit $?
tail -1 "$OUT/parity.log"
for rep in 1 2 3; do
  for v in base prio; do
    for b in 1 2 4 16; do
      case $v in base) E="CDA_RS16_PRIO_MAX=0" ;; prio) E="" ;; esac
      env $E timeout -k 10 200 python -u bench.py --k 512 --batch $b --no-cpu --no-extras --steps 30 --warmup 40 \
        > "$OUT/ab_${v}_b${b}_r${rep}.log" 2>&1 || exit $?
      python - "$OUT/ab_${v}_b${b}_r${rep}.log" "$v" "$b" <<'PY' | tee -a "$OUT/ab.txt"
import json, sys
s = open(sys.argv[1]).read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
st = j.get("stages", {})
b = int(sys.argv[3])
rs = sum(st[x]["avg_ms"] for x in ("rs_q0", "rs_q3") if x in st)
print(sys.argv[2], "batch", b, "ms/sq %.4f" % (j["ms_per_step"] / b), "RS/sq %.4f" % (rs / b))
PY
    done
  done
done
