#!/bin/bash
# Round-3 GPU call "ab": subtrees where the level launches run down to the
# roots (product, CDA_SUBTREE_STOP1=1) against build_var/nost1 over batch
# shapes: k=128 x 16/64/128/256/1024, k=512 x 4/32; parity of the affected shapes.
set -o pipefail
O=gpurun_out/r03ab
mkdir -p $O
B=$GRAFT_REPO_ROOT/celestia-app_amd/build_var
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/test_config4.py tests/test_gpu_parity.py tests/test_variants.py -m gpu > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for i in 1 2; do
  for shape in "128 16" "128 64" "128 128" "128 256" "512 4" "512 32" "128 1024"; do
    set -- $shape
    for v in prod nost1; do
      if [ $v = nost1 ]; then export CDA_LIB=$B/nost1/libcda.so; else unset CDA_LIB; fi
      if [ $2 = 1024 ]; then X=""; else X="--k $1 --batch $2 --distinct $(( $2 < 16 ? $2 : 16 ))"; fi
      timeout -k 10 200 python -u bench.py $X --no-cpu --no-extras --steps 10 --warmup 2 > $O/b.json 2>>$O/ab.err || exit 3
      python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); s=d['stages']; print('k=$1 n=$2 $v', round(d['value'],1), round(d['ms_per_step'],4), round(s['nmt_levels']['avg_ms'],4))" >> $O/ab.txt
    done
  done
done
unset CDA_LIB
cat $O/ab.txt
