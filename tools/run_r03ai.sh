#!/bin/bash
# Round-3 GPU call "ai": tree-top start level (CDA_TOP_FUSE = nodes per tree
# where the fused tree top takes over; auto = 128 for one k=128 square, 32 for
# one k=512 square) on the final build: latency harness, interleaved.
set -o pipefail
O=gpurun_out/r03ai
mkdir -p $O
for i in 1 2 3; do
  for v in auto 64 256; do
    if [ $v = auto ]; then unset CDA_TOP_FUSE; else export CDA_TOP_FUSE=$v; fi
    timeout -k 10 120 python -u tools/latency_ab.py >> $O/lat.txt 2>>$O/ab.err || exit 2
  done
done
unset CDA_TOP_FUSE
python3 -c "
import json
for l in open('$O/lat.txt'):
    d=json.loads(l); e=d['env']; print(e.get('CDA_TOP_FUSE','auto'), round(d['k128_ms_median'],4), round(d['k512_ms_median'],4), round(d['k512_ms_min'],4))
"
