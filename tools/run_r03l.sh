#!/bin/bash
# Round-3 GPU call "l": GF(2^16) half kernel with LDS-DMA (plane-major)
# table staging -- parity of k = 256 / 512 (product + the no-DMA variant),
# then interleaved latency A/B product vs -DCDA_RS16_GLDS=0.
set -o pipefail
O=gpurun_out/r03l
mkdir -p $O
V=$GRAFT_REPO_ROOT/celestia-app_amd/build_var/noglds/libcda.so
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py tests/test_variants.py -m gpu -k "512 or 256 or gf16 or full_width" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
CDA_LIB=$V timeout -k 10 200 $T tests/test_gpu_parity.py -m gpu -k "512 or 256 or gf16" > $O/noglds_parity.log 2>&1 || { tail -30 $O/noglds_parity.log; exit 2; }
tail -1 $O/noglds_parity.log
for i in 1 2 3; do
  CDA_LIB=$V CDA_VARIANT=noglds timeout -k 10 120 python -u tools/latency_ab.py >> $O/glds_ab.txt 2>>$O/ab.err || exit 3
  timeout -k 10 120 python -u tools/latency_ab.py >> $O/glds_ab.txt 2>>$O/ab.err || exit 3
done
cat $O/glds_ab.txt
for i in 1 2; do
  for v in prod noglds; do
    if [ $v = noglds ]; then export CDA_LIB=$V; else unset CDA_LIB; fi
    timeout -k 10 200 python -u bench.py --k 512 --batch 4 --distinct 4 --no-cpu --no-extras --steps 20 --warmup 3 > $O/b512x4_${v}_$i.json 2>>$O/ab.err || exit 4
    python3 -c "import json; d=json.loads(open('$O/b512x4_${v}_$i.json').read().strip().splitlines()[-1]); print('k=512 n=4 $v', round(d['value'],1), round(d['ms_per_step'],4), round(d['stages']['rs_q0']['avg_ms'],4), round(d['stages']['rs_q3']['avg_ms'],4))" >> $O/batch_ab.txt
  done
done
unset CDA_LIB
cat $O/batch_ab.txt
