#!/bin/bash
# Round-3 GPU call "j": fused subtree levels (nmt.hip subtree_kernel) --
# parity (k = 256 / 512 squares, the 16-square config-4 variant test, the
# GPU suite), then interleaved A/B CDA_SUBTREE=0 vs default: single-square
# latency (config 2 / 3) and batches of k = 512 (2, 4) and k = 128 (16, 64).
set -o pipefail
O=gpurun_out/r03k
mkdir -p $O
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 200 $T tests/test_gpu_parity.py tests/test_variants.py -m gpu -k "512 or 256 or gf16 or gf8_q0" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 400 $T tests -m gpu -k "config4 or variants or gpu_parity" > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 2; }
tail -1 $O/gpu_tests.log
for i in 1 2 3; do
  CDA_SUBTREE=0 timeout -k 10 120 python -u tools/latency_ab.py >> $O/lat_ab.txt 2>>$O/ab.err || exit 3
  timeout -k 10 120 python -u tools/latency_ab.py >> $O/lat_ab.txt 2>>$O/ab.err || exit 3
done
cat $O/lat_ab.txt
for cfg in "512 2" "512 4" "128 16" "128 64"; do
  set -- $cfg
  for i in 1 2; do
    for S in 0 8; do
      CDA_SUBTREE=$S timeout -k 10 200 python -u bench.py --k $1 --batch $2 --distinct $2 --no-cpu --no-extras --steps 20 --warmup 3 > $O/b_k$1_n$2_s${S}_$i.json 2>>$O/ab.err || exit 4
      python3 -c "import json,sys; d=json.loads(open('$O/b_k$1_n$2_s${S}_$i.json').read().strip().splitlines()[-1]); print('k=$1 n=$2 CDA_SUBTREE=$S', round(d['value'],1), round(d['ms_per_step'],4))" >> $O/batch_ab.txt
    done
  done
done
cat $O/batch_ab.txt
