# r04zb: greedy plan with triples, 12 (product) vs 14 vs 16 signals
# (build_var/t14, t16): GF(2^16) parity of both, k=512 RS per square
set -e
mkdir -p gpurun_out/r04zb
cd $GRAFT_REPO_ROOT
for v in t14 t16; do
  CDA_LIB=$PWD/celestia-app_amd/build_var/$v/libcda.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "gf16 or k512 or 256 or 512 or codec" > gpurun_out/r04zb/parity_$v.log 2>&1 || { tail -5 gpurun_out/r04zb/parity_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r04zb/parity_$v.log)"
done
for rep in 1 2 3; do
  for v in t12 t14 t16; do
    L=$PWD/celestia-app_amd/libcda.so; [ $v != t12 ] && L=$PWD/celestia-app_amd/build_var/$v/libcda.so
    for b in 1 4 16; do
      CDA_LIB=$L timeout -k 10 200 python bench.py --k 512 --batch $b --no-cpu --no-extras --steps 10 > gpurun_out/r04zb/${v}_$b.log 2>&1
      python - $v $b <<'PY'
import json, sys
v, b = sys.argv[1:3]
s = open(f"gpurun_out/r04zb/{v}_{b}.log").read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
st = j.get("stages", {})
print(v, "batch", b, "ms/sq", round(j["ms_per_step"] / int(b), 4), "RS/sq", round(sum(st[k]["avg_ms"] for k in ("rs_q0", "rs_q3") if k in st) / int(b), 4))
PY
    done
  done
done
