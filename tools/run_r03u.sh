#!/bin/bash
# Round-3 GPU call "u": persistent grid for the GF(2^16) half kernel
# (CDA_RS16_PERSIST=1: two workgroups per CU walk the codeword halves, so
# CU partners start every item together) -- parity, latency / batch A/B,
# phase probe in both grid forms.
set -o pipefail
O=gpurun_out/r03u
mkdir -p $O
B=$GRAFT_REPO_ROOT/celestia-app_amd/build_var
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py tests/test_variants.py -m gpu -k "512 or 256 or gf16" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for i in 1 2 3; do
  CDA_RS16_PERSIST=1 timeout -k 10 120 python -u tools/latency_ab.py >> $O/persist_ab.txt 2>>$O/ab.err || exit 2
  timeout -k 10 120 python -u tools/latency_ab.py >> $O/persist_ab.txt 2>>$O/ab.err || exit 2
done
cat $O/persist_ab.txt
for i in 1 2; do
  for v in 0 1; do
    CDA_RS16_PERSIST=$v timeout -k 10 200 python -u bench.py --k 512 --batch 4 --distinct 4 --no-cpu --no-extras --steps 20 --warmup 3 > $O/b_${v}_$i.json 2>>$O/ab.err || exit 3
    python3 -c "import json; d=json.loads(open('$O/b_${v}_$i.json').read().strip().splitlines()[-1]); print('k=512 n=4 persist=$v', round(d['value'],1), round(d['ms_per_step'],4), round(d['stages']['rs_q0']['avg_ms'],4), round(d['stages']['rs_q3']['avg_ms'],4))" >> $O/batch_ab.txt
  done
done
cat $O/batch_ab.txt
for v in 0 1; do
  CDA_RS16_PERSIST=$v CDA_LIB=$B/rs16ph/libcda.so timeout -k 10 120 python -u tools/rs16_phases.py > $O/rs16_phases_p$v.txt 2>>$O/ab.err || exit 4
done
tail -5 $O/rs16_phases_p1.txt
