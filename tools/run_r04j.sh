# r04j: config 4 at N = 8 (128 squares per GPU) -- subtree occupancy / lanes /
# hash-split A/B against the 1024-square step on the same box
set -e
mkdir -p gpurun_out/r04j
cd $GRAFT_REPO_ROOT
P=$PWD/celestia-app_amd/libcda.so
S4=$PWD/celestia-app_amd/build_var/st4/libcda.so
run() {   # name lib batch env...
  local name=$1 lib=$2 b=$3; shift 3
  env CDA_LIB=$lib "$@" timeout -k 10 200 python bench.py --batch $b --no-extras --no-cpu --steps 20 --warmup 5 > gpurun_out/r04j/$name.log 2>&1
  echo "$name b=$b $* $(grep -o '"value": [0-9.]*' gpurun_out/r04j/$name.log | head -1)"
}
WD=$PWD/celestia-app_amd/build_var/wide/libcda.so
CDA_LIB=$WD timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r04j/wide_parity.log 2>&1
tail -1 gpurun_out/r04j/wide_parity.log
for rep in 1 2; do
  for v in "$P 2" "$WD 0" "$WD 1" "$WD 2"; do
    set -- $v
    echo "lib=$(basename $(dirname $1)) wide=$2 $(CDA_LIB=$1 CDA_TOP_WIDE=$2 timeout -k 10 200 python tools/latency_ab.py 2>&1 | tail -1)"
  done
  for w in 0 2; do
    CDA_LIB=$WD CDA_TOP_WIDE=$w timeout -k 10 150 python bench.py --k 512 --batch 1 --no-cpu --no-extras --steps 10 > gpurun_out/r04j/k512_w$w.log 2>&1
    python - $w <<'PY'
import json, sys
s = open(f"gpurun_out/r04j/k512_w{sys.argv[1]}.log").read()
j = json.loads(s[s.index('{"metric'):].splitlines()[0])
print("k512 wide", sys.argv[1], round(j["ms_per_step"], 4), {k: round(x["avg_ms"], 4) for k, x in j.get("stages", {}).items()})
PY
  done
done
for rep in 1 2; do
  run prod_b1024_$rep $P 1024
  run st4_b1024_$rep $S4 1024
  run prod_$rep $P 128
  run prod_split1_$rep $P 128 CDA_HASH_SPLIT=1
  run prod_lanes64k_$rep $P 128 CDA_SUBTREE_LANES=65536
  run st4_$rep $S4 128
  run st4_split1_$rep $S4 128 CDA_HASH_SPLIT=1 CDA_SUBTREE_LANES=262144
  run st4_split1l131k_$rep $S4 128 CDA_HASH_SPLIT=1
done
