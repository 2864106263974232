#!/bin/bash
# Round-3 GPU call "ar": confirmation A/B -- product now without the subtree
# prefetch (three waves per SIMD) against build_var/pf (the prefetching form,
# two waves): one k=512 square x5 and config 4 x3, interleaved.
set -o pipefail
O=gpurun_out/r03ar
mkdir -p $O
B=$GRAFT_REPO_ROOT/celestia-app_amd/build_var
for i in 1 2 3 4 5; do
  for v in nopf pf; do
    if [ $v = pf ]; then export CDA_LIB=$B/pf/libcda.so; else unset CDA_LIB; fi
    export CDA_VARIANT=$v
    timeout -k 10 120 python -u tools/latency_ab.py >> $O/lat.txt 2>>$O/ab.err || exit 2
    if [ $i -le 3 ]; then
      timeout -k 10 200 python -u bench.py --no-cpu --no-extras --steps 10 --warmup 2 > $O/b.json 2>>$O/ab.err || exit 3
      python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); s=d['stages']; print('cfg4 $v', round(d['value'],1), round(d['ms_per_step'],3), round(s['nmt_levels']['avg_ms'],3))" >> $O/ab.txt
    fi
  done
done
unset CDA_LIB CDA_VARIANT
cat $O/ab.txt
python3 -c "
import json
for l in open('$O/lat.txt'):
    d=json.loads(l); e=d['env']; print(e.get('CDA_VARIANT'), round(d['k128_ms_median'],4), round(d['k512_ms_median'],4), round(d['k512_ms_min'],4))
"
