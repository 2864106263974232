#!/bin/bash
# GPU-box A/B (round 5): k = 512 RS with masks derived at use (build_var/bs16lm)
# against the product kernel, and the leaf overlap (CDA_LEAF_OVERLAP) against
# the serial schedule: single-square latency (config 2 / 3, tools/latency_ab.py,
# packed entry) and k = 512 batches (bench.py, in place).  gpurun_out/<tag>/.
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
summ() {
python - "$1" "$2" "$3" <<'PY' | tee -a "$OUT/ab.txt"
import json, sys
s = open(sys.argv[1]).read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
st = j.get("stages", {})
b = int(sys.argv[3])
rs = sum(st[x]["avg_ms"] for x in ("rs_q0", "rs_q3") if x in st)
print(sys.argv[2], "batch", b, "ms/sq %.4f" % (j["ms_per_step"] / b), "RS/sq %.4f" % (rs / b),
      {k: round(v["avg_ms"], 3) for k, v in st.items()})
PY
}
for rep in 1 2; do
  for v in base lm ovl; do
    for b in 1 4; do
      case $v in
        base) E="CDA_LEAF_OVERLAP=0" ;;
        lm) E="CDA_LIB=$PWD/celestia-app_amd/build_var/bs16lm/libcda.so" ;;
        ovl) E="CDA_LEAF_OVERLAP=16" ;;
      esac
      env $E timeout -k 10 200 python -u bench.py --k 512 --batch $b --no-cpu --no-extras --steps 20 \
        > "$OUT/ab_${v}_b${b}_r${rep}.log" 2>&1 || exit $?
      summ "$OUT/ab_${v}_b${b}_r${rep}.log" $v $b
    done
  done
  for v in 0 16; do
    CDA_LEAF_OVERLAP=$v timeout -k 10 200 python -u tools/latency_ab.py > "$OUT/lat_${v}_r${rep}.log" 2>&1 || exit $?
    echo "overlap=$v $(tail -1 $OUT/lat_${v}_r${rep}.log)" | tee -a "$OUT/ab.txt"
  done
done
