set -o pipefail
mkdir -p gpurun_out/stp
for r in 1 2; do
for v in base p3 p2; do
  if [ $v = base ]; then L=celestia-app_amd/libcda.so; else L=tools/var/rs16_$v/libcda.so; fi
  CDA_BENCH_NOCHECK=1 CDA_LIB=$PWD/$L timeout -k 10 150 python bench.py --k 512 --batch 4 --distinct 1 --no-cpu --no-extras --steps 10 --warmup 3 > gpurun_out/stp/$v.log 2>&1 || { tail -5 gpurun_out/stp/$v.log; exit 2; }
  python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
s = open(f"gpurun_out/stp/{v}.log").read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
print(v, {k: round(x["avg_ms"], 3) for k, x in j["stages"].items() if k.startswith("rs")}, flush=True)
PY
done
done
