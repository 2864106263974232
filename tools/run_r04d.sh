# r04d: bitsliced GF(2^16) variants A/B (k = 512): product (2 waves/SIMD, 2 chunks), bs3 (3 waves/SIMD, 1 chunk),
# bs2c1 (2 waves, 1 chunk), v_perm form
set -e
mkdir -p gpurun_out/r04d
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
for v in bs3 bs3pf bs2pf vperm; do
  L=$PWD/celestia-app_amd/libcda.so; X=1
  [ $v = bs3 ] && L=$PWD/celestia-app_amd/build_var/bs3/libcda.so
  [ $v = bs3pf ] && L=$PWD/celestia-app_amd/build_var/bs3pf/libcda.so
  [ $v = bs2pf ] && L=$PWD/celestia-app_amd/build_var/bs2pf/libcda.so
  [ $v = vperm ] && X=0
  for b in 1 4; do
    CDA_LIB=$L CDA_RS16_BS=$X timeout -k 10 150 python bench.py --k 512 --batch $b --no-cpu --no-extras --steps 20 > gpurun_out/r04d/ab_${v}_$b.log 2>&1
    python - "$v" "$b" <<'PY'
import json, sys
v, b = sys.argv[1:3]
s = open(f"gpurun_out/r04d/ab_{v}_{b}.log").read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
st = j.get("stages", {})
print(v, "batch", b, round(j["ms_per_step"] / int(b), 4), "ms/sq  RS", round((st["rs_q0"]["avg_ms"] + st["rs_q3"]["avg_ms"]) / int(b), 4), {k: round(x["avg_ms"], 3) for k, x in st.items()})
PY
  done
done
done
