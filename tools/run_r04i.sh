# r04i: D2H two-stream A/B (host pipeline, 1024 squares) + kernel traces of the
# 128-square (config 4 at N = 8) and 1024-square steps
set -e
mkdir -p gpurun_out/r04i
cd $GRAFT_REPO_ROOT
for v in 1 0 1 0; do echo "d2h2=$v"; CDA_HOST_D2H2=$v timeout -k 10 200 python tools/host_pipe_run.py 1024 2 2>&1 | grep eds=True; done > gpurun_out/r04i/pipe2.txt 2>&1
cat gpurun_out/r04i/pipe2.txt
cd /tmp && export TMPDIR=/tmp
for b in 128 1024; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04i/prof_b$b -o b$b -- python3 $GRAFT_REPO_ROOT/bench.py --batch $b --no-extras --no-cpu --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r04i/prof_b$b.log 2>&1
done
cd $GRAFT_REPO_ROOT
CDA_LIB=$PWD/celestia-app_amd/build_var/wfold/libcda.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "gf16 or k512 or codec_encode" > gpurun_out/r04i/wfold_parity.log 2>&1
tail -2 gpurun_out/r04i/wfold_parity.log
for rep in 1 2; do
for v in prod stag20 stag35 wfold; do
  L=$PWD/celestia-app_amd/libcda.so
  [ $v != prod ] && L=$PWD/celestia-app_amd/build_var/$v/libcda.so
  for b in 1 4; do
    CDA_LIB=$L timeout -k 10 150 python bench.py --k 512 --batch $b --no-cpu --no-extras --steps 10 > gpurun_out/r04i/st_${v}_$b.log 2>&1
    python - "$v" "$b" <<'PY'
import json, sys
v, b = sys.argv[1:3]
s = open(f"gpurun_out/r04i/st_{v}_{b}.log").read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
st = j.get("stages", {})
print(v, "batch", b, round(j["ms_per_step"] / int(b), 4), "ms/sq  RS", round((st["rs_q0"]["avg_ms"] + st["rs_q3"]["avg_ms"]) / int(b), 4), {k: round(x["avg_ms"], 3) for k, x in st.items()})
PY
  done
done
done
for rep in 1 2; do
for v in prod st4; do
  L=$PWD/celestia-app_amd/libcda.so
  [ $v != prod ] && L=$PWD/celestia-app_amd/build_var/$v/libcda.so
  for b in 1 4; do
    CDA_LIB=$L timeout -k 10 150 python bench.py --k 512 --batch $b --no-cpu --no-extras --steps 10 > gpurun_out/r04i/sub_${v}_$b.log 2>&1
    python - "$v" "$b" <<'PY'
import json, sys
v, b = sys.argv[1:3]
s = open(f"gpurun_out/r04i/sub_{v}_{b}.log").read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
st = j.get("stages", {})
print("subtree", v, "batch", b, round(j["ms_per_step"] / int(b), 4), "ms/sq", {k: round(x["avg_ms"], 3) for k, x in st.items()})
PY
  done
done
done
CDA_LIB=$PWD/celestia-app_amd/build_var/st4/libcda.so timeout -k 10 200 python bench.py --no-cpu --no-extras --steps 5 > gpurun_out/r04i/sub_st4_k128.log 2>&1
grep -o '"value": [0-9.]*' gpurun_out/r04i/sub_st4_k128.log | head -1
