# r04a: bitsliced GF(2^16) encoder -- parity tests, A/B against the v_perm form, kernel trace
set -e
mkdir -p gpurun_out/r04a
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "gf16 or k512 or inplace or codec or split or random_square or linear" > gpurun_out/r04a/par16.log 2>&1 || { tail -30 gpurun_out/r04a/par16.log; exit 1; }
tail -2 gpurun_out/r04a/par16.log
for v in 1 0 1 0; do
  for b in 1 4; do
    CDA_RS16_BS=$v timeout -k 10 150 python bench.py --k 512 --batch $b --no-cpu --no-extras --steps 20 > gpurun_out/r04a/ab_${v}_$b.log 2>&1
    python - "$v" "$b" <<'PY'
import json, sys
v, b = sys.argv[1:3]
s = open(f"gpurun_out/r04a/ab_{v}_{b}.log").read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
print("bs" if v == "1" else "vperm", "batch", b, round(j["value"], 1), "sq/s", round(j["ms_per_step"] / int(b), 4), "ms/sq",
      {k: round(x["avg_ms"], 3) for k, x in j.get("stages", {}).items()})
PY
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04a/prof -o k512 -- python3 $GRAFT_REPO_ROOT/bench.py --k 512 --batch 1 --no-cpu --no-extras --steps 10 > $GRAFT_REPO_ROOT/gpurun_out/r04a/prof.log 2>&1
find $GRAFT_REPO_ROOT/gpurun_out/r04a/prof -name "*kernel_stats.csv" | head -1 | xargs head -12
