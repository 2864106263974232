#!/bin/bash
# Round-3 GPU call "az": hash split at config 4's N = 2 / N = 1 shard sizes
# (512 / 1024 squares per GPU; auto = one stream above 256 squares) vs two streams.
set -o pipefail
O=gpurun_out/r03az
mkdir -p $O
for i in 1 2; do
  for n in 512 1024; do
    for split in auto 2; do
      if [ $split = auto ]; then unset CDA_HASH_SPLIT; else export CDA_HASH_SPLIT=$split; fi
      timeout -k 10 200 python -u bench.py --batch $n --distinct 16 --no-cpu --no-extras --steps 8 --warmup 2 > $O/b.json 2>>$O/ab.err || exit 3
      python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('n=$n split=$split', round(d['value'],1), round(d['ms_per_step'],3))" >> $O/ab.txt
    done
  done
done
unset CDA_HASH_SPLIT
cat $O/ab.txt
