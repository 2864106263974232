#!/bin/bash
# Round-3 GPU call "an": CDA_RS_OVERLAP=1 (GF(2^16) squares: the Q0 launch's
# row codewords on a low-priority stream, columns then Q3 on the call's
# stream) -- parity with the knob on, latency and k=512 batch A/B.
set -o pipefail
O=gpurun_out/r03an
mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
CDA_RS_OVERLAP=1 timeout -k 10 400 $T tests/test_gpu_parity.py tests/test_config4.py -m gpu > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for i in 1 2 3; do
  for v in 0 1; do
    CDA_RS_OVERLAP=$v timeout -k 10 120 python -u tools/latency_ab.py >> $O/lat.txt 2>>$O/ab.err || exit 2
  done
done
for i in 1 2; do
  for v in 0 1; do
    CDA_RS_OVERLAP=$v timeout -k 10 200 python -u bench.py --k 512 --batch 4 --distinct 4 --no-cpu --no-extras --steps 20 --warmup 3 > $O/b.json 2>>$O/ab.err || exit 3
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('k=512 n=4 overlap=$v', round(d['value'],1), round(d['ms_per_step'],4))" >> $O/batch_ab.txt
  done
done
cat $O/batch_ab.txt
python3 -c "
import json
for l in open('$O/lat.txt'):
    d=json.loads(l); e=d['env']; print(e.get('CDA_RS_OVERLAP'), round(d['k128_ms_median'],4), round(d['k512_ms_median'],4), round(d['k512_ms_min'],4))
"
