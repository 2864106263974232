#!/bin/bash
# Round-3 GPU call "au": subtree lane target 262144 for trees of >= 1024
# leaves (product) against the old uniform 131072 (CDA_SUBTREE_LANES=131072):
# k=512 x1 latency, k=512 x2 / x4 batches; parity of the k=512 tests.
set -o pipefail
O=gpurun_out/r03au
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_variants.py -m gpu -k "512 or gf16" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for i in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then export CDA_SUBTREE_LANES=131072; else unset CDA_SUBTREE_LANES; fi
    export CDA_VARIANT=$v
    timeout -k 10 120 python -u tools/latency_ab.py >> $O/lat.txt 2>>$O/ab.err || exit 2
    for n in 2 4; do
      timeout -k 10 200 python -u bench.py --k 512 --batch $n --distinct $n --no-cpu --no-extras --steps 10 --warmup 2 > $O/b.json 2>>$O/ab.err || exit 3
      python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('k=512 n=$n $v', round(d['value'],1), round(d['ms_per_step'],4))" >> $O/ab.txt
    done
  done
done
unset CDA_SUBTREE_LANES CDA_VARIANT
cat $O/ab.txt
python3 -c "
import json
for l in open('$O/lat.txt'):
    d=json.loads(l); e=d['env']; print(e.get('CDA_VARIANT'), round(d['k128_ms_median'],4), round(d['k512_ms_median'],4), round(d['k512_ms_min'],4))
"
