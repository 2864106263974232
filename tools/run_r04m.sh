# r04m: fused data root in the tree top (tickets), wide tree top, 4-wave
# subtree selection -- GPU suite, then same-box A/B of the knobs
set -e
mkdir -p gpurun_out/r04m
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04m/gpu_tests.log 2>&1 || { tail -5 gpurun_out/r04m/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r04m/gpu_tests.log
for rep in 1 2; do
  for e in "" "CDA_TOP_ROOT=0" "CDA_TOP_ROOT=0 CDA_TOP_WIDE=0"; do
    echo "lat [$e] $(env $e timeout -k 10 200 python tools/latency_ab.py 2>&1 | tail -1)"
  done
  for e in "" "CDA_SUBTREE_WAVES=3"; do
    env $e timeout -k 10 200 python bench.py --batch 128 --no-extras --no-cpu --steps 20 --warmup 5 > gpurun_out/r04m/b128_$rep.log 2>&1
    echo "b128 [$e] $(grep -o '"value": [0-9.]*' gpurun_out/r04m/b128_$rep.log | head -1)"
  done
  timeout -k 10 200 python bench.py --batch 1024 --no-extras --no-cpu --steps 10 --warmup 3 > gpurun_out/r04m/b1024_$rep.log 2>&1
  echo "b1024 $(grep -o '"value": [0-9.]*' gpurun_out/r04m/b1024_$rep.log | head -1)"
done
