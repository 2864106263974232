#!/bin/bash
# Round-3 GPU call "v": same-box A/B of the looped half kernel
# (grid (2*ncw, n), one item per workgroup; build_var/loop) against the product.
set -o pipefail
O=gpurun_out/r03v
mkdir -p $O
B=$GRAFT_REPO_ROOT/celestia-app_amd/build_var
for i in 1 2 3; do
  for v in prod loop; do
    if [ $v = loop ]; then export CDA_LIB=$B/loop/libcda.so; else unset CDA_LIB; fi
    timeout -k 10 200 python -u bench.py --k 512 --batch 4 --distinct 4 --no-cpu --no-extras --steps 20 --warmup 3 > $O/b_${v}_$i.json 2>>$O/ab.err || exit 3
    python3 -c "import json; d=json.loads(open('$O/b_${v}_$i.json').read().strip().splitlines()[-1]); print('k=512 n=4 $v', round(d['value'],1), round(d['ms_per_step'],4), round(d['stages']['rs_q0']['avg_ms'],4), round(d['stages']['rs_q3']['avg_ms'],4))" >> $O/batch_ab.txt
  done
done
unset CDA_LIB
cat $O/batch_ab.txt
