# r04t: GF(2^16) RS as columns + Q3 on a high-priority stream beside the rows
# (CDA_RS16_SPLIT=1) vs the two-launch form (=0): parity, then k=512 wall times
set -e
mkdir -p gpurun_out/r04t
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "gf16 or k512 or 256 or 512 or batch" > gpurun_out/r04t/parity.log 2>&1 || { tail -5 gpurun_out/r04t/parity.log; exit 1; }
tail -1 gpurun_out/r04t/parity.log
for rep in 1 2 3; do
  for v in 1 0; do
    echo "split=$v $(CDA_RS16_SPLIT=$v timeout -k 10 200 python tools/latency_ab.py 2>&1 | tail -1)"
    for b in 4 16; do
      CDA_RS16_SPLIT=$v timeout -k 10 200 python bench.py --k 512 --batch $b --no-cpu --no-extras --steps 10 > gpurun_out/r04t/b${b}_$v.log 2>&1
      echo "split=$v batch $b $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r04t/b${b}_$v.log | head -1)"
    done
  done
done
