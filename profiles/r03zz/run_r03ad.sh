#!/bin/bash
# Round-3 GPU call "ad": the default bench line against the final build's
# fixed-shape PMC summary (profiles/r03zz_pmc.json), twice.
set -o pipefail
O=gpurun_out/r03ad
mkdir -p $O
for i in 1 2; do
  timeout -k 10 400 python -u bench.py > $O/bench_$i.json 2> $O/bench_$i.err || { tail -20 $O/bench_$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['extras']['latency_single_square_ms'], d['extras']['k512']['ms_per_square'])"
done
