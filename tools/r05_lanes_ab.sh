#!/bin/bash
# GPU-box A/B (round 5): the subtree launch's lane target (CDA_SUBTREE_LANES)
# at config 4's per-GPU shard sizes (128 squares = N = 8, 256 = N = 4, 64),
# with and without one hash stream; and the k = 512 Q0 launch with its column
# codewords first (build_var/colsfirst).
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
one() {   # <name> <batch> <env...>
  local v=$1 b=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --batch $b --no-cpu --no-extras --steps 20 > "$OUT/${v}_b${b}.log" 2>&1 || return $?
  python - "$OUT/${v}_b${b}.log" $v $b <<'PY' | tee -a "$OUT/ab.txt"
import json, sys
s = open(sys.argv[1]).read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
st = j.get("stages", {})
print(sys.argv[2], "batch", sys.argv[3], "sq/s %.1f" % j["value"], "ms/step %.3f" % j["ms_per_step"],
      "parity", j.get("parity", {}).get("matched"), {k: round(v["avg_ms"], 3) for k, v in st.items()})
PY
}
for rep in 1 2; do
  one b1024 1024 CDA_X=0 || exit $?
  for b in 128 256 64; do
    one base $b CDA_X=0 || exit $?
    one sl256k $b CDA_SUBTREE_LANES=262144 || exit $?
    one sl512k_hs1 $b CDA_SUBTREE_LANES=524288 CDA_HASH_SPLIT=1 || exit $?
  done
  for b in 1 4; do
    for v in base colsfirst; do
      E="CDA_X=0"; [ $v = colsfirst ] && E="CDA_LIB=$PWD/celestia-app_amd/build_var/colsfirst/libcda.so"
      env $E timeout -k 10 200 python -u bench.py --k 512 --batch $b --no-cpu --no-extras --steps 20 > "$OUT/k512_${v}_b${b}.log" 2>&1 || exit $?
      python - "$OUT/k512_${v}_b${b}.log" $v $b <<'PY' | tee -a "$OUT/ab.txt"
import json, sys
s = open(sys.argv[1]).read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
st = j.get("stages", {}); b = int(sys.argv[3])
rs = sum(st[x]["avg_ms"] for x in ("rs_q0", "rs_q3") if x in st)
print("k512", sys.argv[2], "batch", b, "ms/sq %.4f" % (j["ms_per_step"] / b), "RS/sq %.4f" % (rs / b),
      {k: round(v["avg_ms"], 3) for k, v in st.items()})
PY
    done
  done
done
