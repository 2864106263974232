#!/bin/bash
# Round-3 GPU call "ao": the N = 8 / N = 4 shard shapes of config 4 (128 and
# 256 squares per GPU): hash split (auto = 2 streams at <= 256 squares) x
# subtree lane target (131072 default; 65536 lets one stream hash whole trees).
set -o pipefail
O=gpurun_out/r03ao
mkdir -p $O
for i in 1 2; do
  for n in 128 256; do
    for split in auto 1; do
      for L in 131072 65536; do
        if [ $split = auto ]; then unset CDA_HASH_SPLIT; else export CDA_HASH_SPLIT=$split; fi
        export CDA_SUBTREE_LANES=$L
        timeout -k 10 200 python -u bench.py --batch $n --distinct 16 --no-cpu --no-extras --steps 10 --warmup 2 > $O/b.json 2>>$O/ab.err || exit 3
        python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('n=$n split=$split lanes=$L', round(d['value'],1), round(d['ms_per_step'],4))" >> $O/ab.txt
      done
    done
  done
done
unset CDA_HASH_SPLIT CDA_SUBTREE_LANES
cat $O/ab.txt
