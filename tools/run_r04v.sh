# r04v: k=512 one square: stage-pass RS time and wall time with the split RS
# (CDA_RS16_SPLIT=1) vs Q0 then Q3 (=0), 3 interleaved reps
set -e
mkdir -p gpurun_out/r04v
cd $GRAFT_REPO_ROOT
for rep in 1 2 3; do
  for v in 1 0; do
    CDA_RS16_SPLIT=$v timeout -k 10 200 python bench.py --k 512 --batch 1 --no-cpu --no-extras --steps 20 > gpurun_out/r04v/s${v}_$rep.log 2>&1
    python - $v $rep <<'PY'
import json, sys
v, rep = sys.argv[1:3]
s = open(f"gpurun_out/r04v/s{v}_{rep}.log").read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
st = j.get("stages", {})
print("split", v, "wall ms", round(j["ms_per_step"], 4), "RS stage", round(sum(st[k]["avg_ms"] for k in ("rs_q0", "rs_q3") if k in st), 4), {k: round(x["avg_ms"], 4) for k, x in st.items()})
PY
  done
done
