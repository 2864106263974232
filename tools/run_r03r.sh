#!/bin/bash
# Round-3 GPU call "r": per-GPU rate of config 4's shard sizes at N = 8 / 4 / 2
# / 1 (128 / 256 / 512 / 1024 squares per step), bench without extras.
set -o pipefail
O=gpurun_out/r03r
mkdir -p $O
for B in 128 256 512 1024 128; do
  timeout -k 10 300 python -u bench.py --batch $B --distinct $B --no-cpu --no-extras --steps 20 --warmup 3 > $O/b$B.json 2>>$O/err.log || exit 1
  python3 -c "import json; d=json.loads(open('$O/b$B.json').read().strip().splitlines()[-1]); print($B, round(d['value'],1), round(d['ms_per_step'],4), {k: round(v['avg_ms'],4) for k,v in d['stages'].items()})" | tee -a $O/shards.txt
done
