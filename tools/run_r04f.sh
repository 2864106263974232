# r04f: bitsliced GF(2^16) with pair signals (3 waves/SIMD) vs v_perm form, + gf16 parity tests
set -e
mkdir -p gpurun_out/r04f
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "gf16 or k512 or inplace or codec or split or random_square or linear" > gpurun_out/r04f/par16.log 2>&1 || { tail -30 gpurun_out/r04f/par16.log; exit 1; }
tail -1 gpurun_out/r04f/par16.log
for rep in 1 2; do
for v in prod vperm; do
  X=1; [ $v = vperm ] && X=0
  for b in 1 4 16; do
    CDA_RS16_BS=$X timeout -k 10 150 python bench.py --k 512 --batch $b --no-cpu --no-extras --steps 10 > gpurun_out/r04f/ab_${v}_$b.log 2>&1
    python - "$v" "$b" <<'PY'
import json, sys
v, b = sys.argv[1:3]
s = open(f"gpurun_out/r04f/ab_{v}_{b}.log").read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
st = j.get("stages", {})
print(v, "batch", b, round(j["ms_per_step"] / int(b), 4), "ms/sq  RS", round((st["rs_q0"]["avg_ms"] + st["rs_q3"]["avg_ms"]) / int(b), 4), {k: round(x["avg_ms"], 3) for k, x in st.items()})
PY
  done
done
done
