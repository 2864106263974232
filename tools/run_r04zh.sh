# r04zh: persistent ticketed GF(2^16) extension (variant library, tools/probes/rs16_ticket_launch.patch form C): parity, then A/B
set -e
mkdir -p gpurun_out/r04zh
cd $GRAFT_REPO_ROOT
export CDA_LIB=$GRAFT_REPO_ROOT/celestia-app_amd/build_var/ticket/libcda.so
timeout -k 10 300 python -u -m pytest tests/test_rs16_ticket_probe.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r04zh/tests.log 2>&1 || { tail -30 gpurun_out/r04zh/tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r04zh/tests.log | tail -2
show() {
python - "$1" "$2" <<'PY'
import json, sys
s = open(sys.argv[1]).read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
st = j["stages"]
print(sys.argv[2], "ms/step %.4f" % j["ms_per_step"], " ".join("%s %.4f" % (k, v["avg_ms"]) for k, v in st.items()))
PY
}
for b in 1 16; do
  for pass in 1 2; do
    for t in 1 0; do
      CDA_RS16_TICKET=$t timeout -k 10 200 python bench.py --k 512 --batch $b --distinct 1 --no-cpu --no-extras --steps 20 --warmup 3 > gpurun_out/r04zh/b${b}_t${t}_p${pass}.log 2>&1 || { tail -5 gpurun_out/r04zh/b${b}_t${t}_p${pass}.log; exit 1; }
      show gpurun_out/r04zh/b${b}_t${t}_p${pass}.log "batch $b ticket=$t pass $pass"
    done
  done
done
