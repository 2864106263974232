# r04o: fused data root fixed (no second data-root pass) -- GPU suite, latency
# A/B (fused / CDA_TOP_ROOT=0 / neither wide nor fused), b128 subtree waves A/B
set -e
mkdir -p gpurun_out/r04o
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04o/gpu_tests.log 2>&1 || { tail -5 gpurun_out/r04o/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04o/gpu_tests.log
for rep in 1 2 3; do
  for e in "" "CDA_TOP_ROOT=0" "CDA_TOP_ROOT=0 CDA_TOP_WIDE=0"; do
    echo "lat [$e] $(env $e timeout -k 10 200 python tools/latency_ab.py 2>&1 | tail -1)"
  done
done
for rep in 1 2 3; do
  for e in "CDA_SUBTREE_WAVES=0" "CDA_SUBTREE_WAVES=3"; do
    env $e timeout -k 10 200 python bench.py --batch 128 --no-extras --no-cpu --steps 20 --warmup 5 > gpurun_out/r04o/b128_$rep.log 2>&1
    echo "b128 [$e] $(grep -o '"value": [0-9.]*' gpurun_out/r04o/b128_$rep.log | head -1)"
  done
done
