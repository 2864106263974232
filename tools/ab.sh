#!/bin/bash
# Parametrised interleaved A/B of bench.py (GPU box), replacing the round-5
# one-off r05_*_ab.sh scripts.  Usage:
#   tools/ab.sh TAG ROUNDS "BENCH ARGS" "ENV A" "ENV B" ["ENV C" ...]
# Each variant is an environment string (e.g. "CDA_LIB=celestia-app_amd/libcda_test.so CDA_RS8_FUSED=0");
# variants run interleaved ROUNDS times; every run's JSON line goes to
# gpurun_out/TAG/<variant index>_<round>.json and a summary (value, ms_per_step,
# stage ms) to gpurun_out/TAG/ab.txt.  Each run has its own time limit; the
# script stops at the first failing run.
set -u
tag=$1; rounds=$2; args=$3; shift 3
out=gpurun_out/$tag
mkdir -p "$out"
: > "$out/ab.txt"
for r in $(seq 1 "$rounds"); do
  i=0
  for v in "$@"; do
    f="$out/${i}_${r}.json"
    if ! env $v timeout -k 10 300 python3 bench.py $args > "$f" 2> "$out/${i}_${r}.err"; then
      echo "variant $i round $r failed: $v" | tee -a "$out/ab.txt"
      exit 1
    fi
    python3 - "$f" "$i" "$v" >> "$out/ab.txt" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
st = d.get("stages", {})
stages = " ".join(f"{k}={v['avg_ms']:.3f}" for k, v in st.items())
k5 = d.get("extras", {}).get("k512", {})
extra = f" k512={k5['ms_per_square']:.3f}ms" if "ms_per_square" in k5 else ""
print(f"[{sys.argv[2]}] {d['value']:.1f} sq/s {d['ms_per_step']:.3f} ms/step parity {d['parity']['matched']}/{d['parity']['checked']} | {stages}{extra} | {sys.argv[3]}")
PY
    i=$((i+1))
  done
done
cat "$out/ab.txt"
