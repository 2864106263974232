#!/bin/bash
# Round-3 GPU call "p": subtree launches sized for two waves per SIMD
# (CDA_SUBTREE_LANES, default 131072), then per-level launches to the tree
# top.  Parity, then A/B: single squares (lanes 65536 = round-3's first form /
# default / CDA_SUBTREE=0) and batches (default vs CDA_SUBTREE=0).
set -o pipefail
O=gpurun_out/r03p
mkdir -p $O
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py tests/test_variants.py tests/test_config4.py -m gpu -k "not all_1024 and not multi_gpu" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for i in 1 2 3; do
  CDA_SUBTREE_LANES=65536 timeout -k 10 120 python -u tools/latency_ab.py >> $O/lat_ab.txt 2>>$O/ab.err || exit 2
  timeout -k 10 120 python -u tools/latency_ab.py >> $O/lat_ab.txt 2>>$O/ab.err || exit 2
  CDA_SUBTREE=0 timeout -k 10 120 python -u tools/latency_ab.py >> $O/lat_ab.txt 2>>$O/ab.err || exit 2
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
