#!/bin/bash
# GPU-box A/B of the subtree kernel's occupancy (round 5): product (3 waves
# per SIMD, 141 VGPRs) against build_var/sub4 (the same source with
# amdgpu_waves_per_eu(4): 128 VGPRs, 9 spilled values).  k = 512 batch 1 / 4
# (262 144-lane launches: 1.33 rounds at 3 waves per SIMD, 1 at 4) and k = 128
# batch 128 / 1024.  Output: gpurun_out/<tag>/ab.txt.
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in 1 2 3; do
  for v in base sub4; do
    for cfg in "512 1" "512 4" "128 128" "128 1024"; do
      set -- $cfg
      case $v in base) E="" ;; sub4) E="CDA_LIB=$PWD/celestia-app_amd/build_var/sub4/libcda.so" ;; esac
      if [ $1 = 512 ]; then S="--steps 30 --warmup 40"; else S="--steps 10 --warmup 3"; fi
      env $E timeout -k 10 200 python -u bench.py --k $1 --batch $2 --no-cpu --no-extras $S \
        > "$OUT/ab_${v}_k$1_b$2_r${rep}.log" 2>&1 || exit $?
      python - "$OUT/ab_${v}_k$1_b$2_r${rep}.log" "$v" "$1" "$2" <<'PY' | tee -a "$OUT/ab.txt"
import json, sys
s = open(sys.argv[1]).read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
st = j.get("stages", {})
b = int(sys.argv[4])
print(sys.argv[2], "k", sys.argv[3], "batch", b, "ms/sq %.4f" % (j["ms_per_step"] / b),
      "levels %.4f" % st["nmt_levels"]["avg_ms"], "parity", j.get("parity", {}).get("matched"),
      {k: round(v["avg_ms"], 3) for k, v in st.items()})
PY
    done
  done
done
