# r04b: GPU suite subsets touched this round + host pipeline leg + k=512 A/B
set -e
mkdir -p gpurun_out/r04b
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_comm_faults.py tests/test_config4.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04b/tests.log 2>&1 || { tail -40 gpurun_out/r04b/tests.log; exit 1; }
tail -3 gpurun_out/r04b/tests.log
timeout -k 10 600 python bench.py --no-cpu --steps 10 > gpurun_out/r04b/bench.log 2>&1 || { tail -30 gpurun_out/r04b/bench.log; exit 1; }
python - <<'PY'
import json
s = open("gpurun_out/r04b/bench.log").read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
print("headline", round(j["value"]), "ms/step", round(j["ms_per_step"], 2))
e = j["extras"]
print("k512", {k: e["k512"].get(k) for k in ("ms_per_square", "data_root_matches_oracle")}, e["k512"].get("rs_roofline", {}).get("ms_per_square"))
print("host_config4", json.dumps(e.get("host_buffers_config4"))[:900])
print("host16", json.dumps(e.get("host_buffers"))[:400])
print("lat", e.get("latency_single_square_ms"))
PY
