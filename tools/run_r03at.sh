#!/bin/bash
# Round-3 GPU call "at": one k=512 square, subtree lane target 131072 (16-leaf
# subtrees + one level launch) vs 262144 (8-leaf subtrees + two level
# launches), interleaved x6 on the HEAD build.
set -o pipefail
O=gpurun_out/r03at
mkdir -p $O
for i in 1 2 3 4 5 6; do
  for L in 131072 262144; do
    CDA_SUBTREE_LANES=$L timeout -k 10 120 python -u tools/latency_ab.py >> $O/lat.txt 2>>$O/ab.err || exit 2
  done
done
python3 -c "
import json
for l in open('$O/lat.txt'):
    d=json.loads(l); e=d['env']; print(e.get('CDA_SUBTREE_LANES'), round(d['k128_ms_median'],4), round(d['k512_ms_median'],4), round(d['k512_ms_min'],4))
"
