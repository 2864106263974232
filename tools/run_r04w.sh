# r04w: config-4 128- and 256-square shards: staggered hash parts
# (CDA_HASH_STAGGER=1, 2 or 4 parts) vs the default (2 parts side by side);
# parity of the 256-square submission with stagger on; then r04v (RS split A/B)
set -e
mkdir -p gpurun_out/r04w
cd $GRAFT_REPO_ROOT
CDA_HASH_STAGGER=1 CDA_HASH_SPLIT=4 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_config4.py tests/test_gpu_parity.py -k "256 or batch or two_streams" > gpurun_out/r04w/parity.log 2>&1 || { tail -5 gpurun_out/r04w/parity.log; exit 1; }
tail -1 gpurun_out/r04w/parity.log
for rep in 1 2 3; do
  for v in "CDA_HASH_STAGGER=0" "CDA_HASH_STAGGER=1" "CDA_HASH_STAGGER=1 CDA_HASH_SPLIT=4" "CDA_HASH_STAGGER=0 CDA_HASH_SPLIT=4"; do
    env $v timeout -k 10 200 python bench.py --batch 128 --no-extras --no-cpu --steps 20 --warmup 5 > gpurun_out/r04w/b128.log 2>&1
    echo "b128 [$v] $(grep -o '"value": [0-9.]*' gpurun_out/r04w/b128.log | head -1)"
  done
done
bash tools/run_r04v.sh
