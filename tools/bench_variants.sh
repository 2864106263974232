#!/bin/bash
# Bench every celestia-app_amd/variants/libcda_*.so (tuning sweeps; run via gpurun).
set -o pipefail
mkdir -p gpurun_out
for so in celestia-app_amd/variants/libcda_*.so; do
  n=$(basename $so .so)
  CDA_BENCH_NOCHECK=1 CDA_LIB=$PWD/$so timeout -k 10 120 python bench.py --no-cpu --no-extras --steps 10 --warmup 2 "$@" > gpurun_out/var_$n.json 2> gpurun_out/var_$n.err || exit 1
  python - "$n" gpurun_out/var_$n.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
st={k:round(v["avg_ms"],3) for k,v in d["stages"].items()}
print(sys.argv[1], round(d["value"],1), st)
PY
done
