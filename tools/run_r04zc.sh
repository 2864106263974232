# r04zc: host leg with the bidirectional line beside it; SDMA copies vs blit-kernel copies (HSA_ENABLE_SDMA=0)
set -e
mkdir -p gpurun_out/r04zc
cd $GRAFT_REPO_ROOT
show() {
python - "$1" <<'PY'
import json, sys
s = open(sys.argv[1]).read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
h = j["extras"]["host_buffers_config4"]
print(sys.argv[1], "value", round(j["value"]), {k: round(v, 3) for k, v in h.items() if isinstance(v, float)}, h["parity"])
PY
}
timeout -k 10 600 python bench.py --no-cpu > gpurun_out/r04zc/sdma1.log 2>&1
show gpurun_out/r04zc/sdma1.log
HSA_ENABLE_SDMA=0 timeout -k 10 600 python bench.py --no-cpu > gpurun_out/r04zc/sdma0.log 2>&1
show gpurun_out/r04zc/sdma0.log
timeout -k 10 600 python bench.py --no-cpu > gpurun_out/r04zc/sdma1b.log 2>&1
show gpurun_out/r04zc/sdma1b.log
