set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "gf16 or k512 or inplace or codec or split or random_square" > gpurun_out/par16.log 2>&1
tail -2 gpurun_out/par16.log
for v in base bfs base bfs; do
  if [ $v = base ]; then L=celestia-app_amd/libcda.so; else L=tools/var/rs16_$v/libcda.so; fi
  CDA_LIB=$PWD/$L timeout -k 10 150 python bench.py --k 512 --batch 4 --no-cpu --no-extras --steps 20 > gpurun_out/ab16_$v.log 2>&1
  python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
s = open(f"gpurun_out/ab16_{v}.log").read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
print(v, round(j["value"], 1), "sq/s", {k: round(x["avg_ms"], 3) for k, x in j["stages"].items()})
PY
done
