set -o pipefail
mkdir -p gpurun_out/ab16
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab16/gputests.log 2>&1 || { tail -20 gpurun_out/ab16/gputests.log; exit 1; }
tail -2 gpurun_out/ab16/gputests.log
for v in new prev new prev; do
  if [ $v = new ]; then L=celestia-app_amd/libcda.so; else L=tools/var/rs16_$v/libcda.so; fi
  for B in 1 4; do
  CDA_LIB=$PWD/$L timeout -k 10 150 python bench.py --k 512 --batch $B --distinct 1 --no-cpu --no-extras --steps 10 --warmup 2 > gpurun_out/ab16/$v$B.log 2>&1 || { tail -5 gpurun_out/ab16/$v$B.log; exit 2; }
  python - "$v$B" <<'PY'
import json, sys
v = sys.argv[1]
s = open(f"gpurun_out/ab16/{v}.log").read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
print(v, round(j["value"], 1), "sq/s", round(j["ms_per_step"], 3), "ms/step", {k: round(x["avg_ms"], 3) for k, x in j["stages"].items()}, flush=True)
PY
  done
done
