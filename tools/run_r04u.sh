# r04u: end-of-round check of the committed build: GPU suite, smoke, default bench
set -e
mkdir -p gpurun_out/r04u
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04u/gpu_tests.log 2>&1 || { tail -5 gpurun_out/r04u/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04u/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04u/smoke.log 2>&1 || { tail -5 gpurun_out/r04u/smoke.log; exit 1; }
tail -1 gpurun_out/r04u/smoke.log
timeout -k 10 900 python bench.py > gpurun_out/r04u/bench.log 2>&1
python - <<'PY'
import json
s = open("gpurun_out/r04u/bench.log").read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
ex = j["extras"]
print("value", round(j["value"]), "frac", round(j["roofline"]["frac"], 3), "traffic", j["roofline"].get("traffic"),
      "lat", round(ex["latency_single_square_ms"], 4), "k512", round(ex["k512"]["ms_per_square"], 4),
      "rs", round(ex["k512"]["rs_roofline"]["ms_per_square"], 4), "host4", round(ex["host_buffers_config4"]["eds_to_host_squares_per_s"]))
PY
