# r04q: block-0 schedule helpers in the tree top's levels of <= 32 parents --
# tree-top parity tests, then latency A/B (CDA_TOP_HELPERS=2 default / 1 / 0)
set -e
mkdir -p gpurun_out/r04q
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_dah.py > gpurun_out/r04q/parity.log 2>&1 || { tail -5 gpurun_out/r04q/parity.log; exit 1; }
tail -1 gpurun_out/r04q/parity.log
for rep in 1 2 3; do
  for e in "CDA_TOP_HELPERS=2" "CDA_TOP_HELPERS=1"; do
    echo "lat [$e] $(env $e timeout -k 10 200 python tools/latency_ab.py 2>&1 | tail -1)"
  done
done
