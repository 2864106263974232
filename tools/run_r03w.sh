#!/bin/bash
# Round-3 GPU call "w": nontemporal parity stores in the GF(2^8) encoder
# (build_var/nt, -DCDA_RS8_NT=1) against the product: config 4 bench stages,
# latency, parity of the variant.
set -o pipefail
O=gpurun_out/r03w
mkdir -p $O
B=$GRAFT_REPO_ROOT/celestia-app_amd/build_var
CDA_LIB=$B/nt/libcda.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "128" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for i in 1 2 3; do
  for v in prod nt; do
    if [ $v = nt ]; then export CDA_LIB=$B/nt/libcda.so; else unset CDA_LIB; fi
    timeout -k 10 200 python -u bench.py --no-cpu --no-extras --steps 10 --warmup 2 > $O/b_${v}_$i.json 2>>$O/ab.err || exit 3
    python3 -c "import json; d=json.loads(open('$O/b_${v}_$i.json').read().strip().splitlines()[-1]); s=d['stages']; print('cfg4 $v', round(d['value'],1), round(d['ms_per_step'],3), *[(k, round(s[k]['avg_ms'],3)) for k in ('rs_q0','rs_q3','nmt_leaves','nmt_levels')])" >> $O/ab.txt
  done
done
unset CDA_LIB
cat $O/ab.txt
for i in 1 2; do
  CDA_LIB=$B/nt/libcda.so CDA_VARIANT=nt timeout -k 10 120 python -u tools/latency_ab.py >> $O/lat.txt 2>>$O/ab.err || exit 2
  timeout -k 10 120 python -u tools/latency_ab.py >> $O/lat.txt 2>>$O/ab.err || exit 2
done
cat $O/lat.txt
