#!/bin/bash
# Round-3 GPU call "ae": subtree_kernel at up to 3 waves per SIMD
# (build_var/sw3, 168 VGPRs, 18 spills) against the product (189 VGPRs, two
# waves per SIMD), with 131072 / 262144 lanes per subtree launch: one k=512
# square (latency harness) and config 4.
set -o pipefail
O=gpurun_out/r03ae
mkdir -p $O
B=$GRAFT_REPO_ROOT/celestia-app_amd/build_var
CDA_LIB=$B/sw3/libcda.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_config4.py -m gpu -k "512 or all_1024" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for i in 1 2; do
  for v in prod sw3; do
    for L in 131072 262144; do
      if [ $v = sw3 ]; then export CDA_LIB=$B/sw3/libcda.so; else unset CDA_LIB; fi
      export CDA_SUBTREE_LANES=$L CDA_VARIANT=$v
      timeout -k 10 120 python -u tools/latency_ab.py >> $O/lat.txt 2>>$O/ab.err || exit 2
      timeout -k 10 200 python -u bench.py --no-cpu --no-extras --steps 10 --warmup 2 > $O/b.json 2>>$O/ab.err || exit 3
      python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); s=d['stages']; print('cfg4 $v $L', round(d['value'],1), round(d['ms_per_step'],3), round(s['nmt_levels']['avg_ms'],3))" >> $O/ab.txt
    done
  done
done
unset CDA_LIB CDA_SUBTREE_LANES CDA_VARIANT
cat $O/ab.txt
python3 -c "
import json
for l in open('$O/lat.txt'):
    d=json.loads(l); e=d['env']; print(e.get('CDA_VARIANT'), e.get('CDA_SUBTREE_LANES'), round(d['k512_ms_median'],4), round(d['k512_ms_min'],4), round(d['k128_ms_median'],4))
"
