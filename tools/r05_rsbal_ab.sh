#!/bin/bash
# GPU-box A/B of the k >= 256 in-place RS launch split (round 5; the balanced form was
# not kept, profiles/r05/rs_balance_ab.txt -- the script needs its engine patch): balanced
# (columns + half the Q0 rows, then the other rows + Q3: 1.5 k codewords per
# launch, the product) against CDA_RS_BALANCE=0 (Q0 rows + columns, then Q3).
# Every k = 512 / GF(2^16) GPU test first, then interleaved benches at batch
# 1 / 4 / 16 (warm-up 40 steps).  Output: gpurun_out/<tag>/ab.txt.
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "512 or gf16 or codec or split or linear or repair or pipeline or fault" > "$OUT/parity.log" 2>&1 || exit $?
tail -1 "$OUT/parity.log"
for rep in 1 2 3; do
  for v in bal old; do
    for b in 1 4 16; do
      case $v in bal) E="" ;; old) E="CDA_RS_BALANCE=0" ;; esac
      env $E timeout -k 10 200 python -u bench.py --k 512 --batch $b --no-cpu --no-extras --steps 30 --warmup 40 \
        > "$OUT/ab_${v}_b${b}_r${rep}.log" 2>&1 || exit $?
      python - "$OUT/ab_${v}_b${b}_r${rep}.log" "$v" "$b" <<'PY' | tee -a "$OUT/ab.txt"
import json, sys
s = open(sys.argv[1]).read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
st = j.get("stages", {})
b = int(sys.argv[3])
rs = sum(st[x]["avg_ms"] for x in ("rs_q0", "rs_q3") if x in st)
print(sys.argv[2], "batch", b, "ms/sq %.4f" % (j["ms_per_step"] / b), "RS/sq %.4f" % (rs / b),
      {k: round(v["avg_ms"], 3) for k, v in st.items()})
PY
    done
  done
done
