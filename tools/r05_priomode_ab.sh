#!/bin/bash
# GPU-box A/B (round 5): GF(2^16) wave-priority schemes (CDA_RS16_PRIO_MODE:
# 1 = 2 loading / 0 / 1 storing, the product; 2 = loads only; 3 = 3 / 0 / 3)
# and none (CDA_RS16_PRIO_MAX=0), at k = 512 batch 1 / 4 / 16 with the flag
# applied to every batch (CDA_RS16_PRIO_MAX=64).  Output: gpurun_out/<tag>/.
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
CDA_RS16_PRIO_MODE=3 CDA_RS16_PRIO_MAX=64 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "512 or gf16" > "$OUT/parity.log" 2>&1 || exit $?
tail -1 "$OUT/parity.log"
for rep in 1 2 3; do
  for v in m0 m1 m2 m3; do
    for b in 1 4 16; do
      case $v in
        m0) E="CDA_RS16_PRIO_MAX=0" ;;
        *) E="CDA_RS16_PRIO_MAX=64 CDA_RS16_PRIO_MODE=${v#m}" ;;
      esac
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
