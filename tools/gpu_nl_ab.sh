set -o pipefail
mkdir -p gpurun_out/nl
for v in nl nlbfs; do
  CDA_LIB=$PWD/tools/var/rs16_$v/libcda.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "gf16 or k512 or linear" > gpurun_out/nl/par_$v.log 2>&1 || { echo "PARITY FAIL $v"; tail -20 gpurun_out/nl/par_$v.log; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/nl/par_$v.log)"
done
for r in 1 2; do
for v in base nl nlbfs; do
  if [ $v = base ]; then L=celestia-app_amd/libcda.so; else L=tools/var/rs16_$v/libcda.so; fi
  for B in 1 4; do
  CDA_LIB=$PWD/$L timeout -k 10 150 python bench.py --k 512 --batch $B --distinct 1 --no-cpu --no-extras --steps 10 --warmup 3 > gpurun_out/nl/$v$B.log 2>&1 || { tail -5 gpurun_out/nl/$v$B.log; exit 2; }
  python - "$v$B" <<'PY'
import json, sys
v = sys.argv[1]
s = open(f"gpurun_out/nl/{v}.log").read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
print(v, round(j["value"], 1), "sq/s", round(j["ms_per_step"], 3), "ms/step", {k: round(x["avg_ms"], 3) for k, x in j["stages"].items() if k.startswith("rs")}, flush=True)
PY
  done
done
done
