# r04l: product build (wide tree top, 4-wave subtree selection): GPU suite,
# latency (configs 2/3), config-4 rates at 1024 and 128 squares, k=512 stages
set -e
mkdir -p gpurun_out/r04l
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04l/gpu_tests.log 2>&1
tail -2 gpurun_out/r04l/gpu_tests.log
for rep in 1 2; do
  timeout -k 10 200 python tools/latency_ab.py 2>&1 | tail -1
  for b in 1024 128; do
    timeout -k 10 200 python bench.py --batch $b --no-extras --no-cpu --steps 20 --warmup 5 > gpurun_out/r04l/b${b}_$rep.log 2>&1
    echo "b=$b $(grep -o '"value": [0-9.]*' gpurun_out/r04l/b${b}_$rep.log | head -1)"
  done
  timeout -k 10 150 python bench.py --k 512 --batch 1 --no-cpu --no-extras --steps 10 > gpurun_out/r04l/k512_$rep.log 2>&1
  python - $rep <<'PY'
import json, sys
s = open(f"gpurun_out/r04l/k512_{sys.argv[1]}.log").read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
print("k512", round(j["ms_per_step"], 4), {k: round(x["avg_ms"], 4) for k, x in j.get("stages", {}).items()})
PY
done
