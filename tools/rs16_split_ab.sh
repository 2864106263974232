#!/bin/bash
# GPU-box A/B of the k = 512 encoder's LOW-layer split (round 5): the product
# kernel runs LOW IFFT layer 0 on each pair of units and layer 1 on each quad
# as soon as their loads land, and stores each pair of units as soon as LOW
# FFT is done with it; build_var/split2/libcda.so (-DCDA_BS16_SPLIT2) splits
# only into halves, build_var/nosplit/libcda.so (-DCDA_BS16_NO_SPLIT) not at
# all.  Then a kernel trace of the timed region of each (TRACE=1).  The two
# variants left the product source in round 5: apply
# tools/probes/rs16_split_variants.patch before building them.  Parity of the product build first
# (every k = 512 / GF(2^16) GPU test), then interleaved bench runs at batch
# 1 / 4 / 16.  Output: gpurun_out/<tag>/.
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "512 or gf16 or codec or split or linear or repair" > "$OUT/parity.log" 2>&1 || exit $?
tail -1 "$OUT/parity.log"
for rep in 1 2; do
  for v in ${VARIANTS:-split split2 nosplit}; do
    for b in 1 4 16; do
      case $v in
        split) E="" ;;
        *) E="CDA_LIB=$PWD/celestia-app_amd/build_var/$v/libcda.so" ;;
      esac
      env $E timeout -k 10 200 python -u bench.py --k 512 --batch $b --no-cpu --no-extras --steps 20 \
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
[ "${TRACE:-0}" = 1 ] || exit 0
cd /tmp && export TMPDIR=/tmp
for v in split nosplit; do
  L=""; [ $v = split ] || L="$GRAFT_REPO_ROOT/celestia-app_amd/build_var/$v/libcda.so"
  CDA_LIB=${L:-$GRAFT_REPO_ROOT/celestia-app_amd/libcda.so} timeout -k 10 200 rocprofv3 --kernel-trace --stats \
    -d "$GRAFT_REPO_ROOT/$OUT/trace_$v" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --k 512 --batch 1 --no-cpu \
    --no-extras --steps 40 > "$GRAFT_REPO_ROOT/$OUT/trace_$v.log" 2>&1 || exit $?
done
