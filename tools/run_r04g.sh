# r04g: full GPU suite + default bench (headline, extras incl. host pipeline)
set -e
mkdir -p gpurun_out/r04g
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04g/gputests.log 2>&1 || { tail -40 gpurun_out/r04g/gputests.log; exit 1; }
tail -2 gpurun_out/r04g/gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04g/smoke.log 2>&1 || { tail -20 gpurun_out/r04g/smoke.log; exit 1; }
tail -1 gpurun_out/r04g/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r04g/bench.log 2>&1 || { tail -30 gpurun_out/r04g/bench.log; exit 1; }
python - <<'PY'
import json
s = open("gpurun_out/r04g/bench.log").read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
print("headline", round(j["value"]), "ms/step", round(j["ms_per_step"], 2), "frac", j["roofline"]["frac"])
e = j["extras"]
print("k512", {k: e["k512"].get(k) for k in ("ms_per_square", "data_root_matches_oracle")}, e["k512"].get("rs_roofline", {}).get("ms_per_square"))
print("host_config4", json.dumps(e.get("host_buffers_config4"))[:1200])
print("lat", e.get("latency_single_square_ms"))
PY
