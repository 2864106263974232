#!/bin/bash
# Round-3 GPU call "ay": leaf kernel without the next-block prefetch
# (build_var/lnp: 122 VGPRs, no spills, four waves per SIMD; build_var/lnp5:
# held to 96 VGPRs = five waves, 15 spills) against the product (128 VGPRs,
# 6 spills), config 4, interleaved x3; parity of the variants.
set -o pipefail
O=gpurun_out/r03ay
mkdir -p $O
B=$GRAFT_REPO_ROOT/celestia-app_amd/build_var
for v in lnp lnp5; do
  CDA_LIB=$B/$v/libcda.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_config4.py tests/test_gpu_parity.py -m gpu -k "all_1024 or 128 or 512" >> $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
done
grep -E "passed|failed" $O/parity.log
for i in 1 2 3; do
  for v in prod lnp lnp5; do
    if [ $v = prod ]; then unset CDA_LIB; else export CDA_LIB=$B/$v/libcda.so; fi
    timeout -k 10 200 python -u bench.py --no-cpu --no-extras --steps 10 --warmup 2 > $O/b.json 2>>$O/ab.err || exit 3
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); s=d['stages']; print('cfg4 $v', round(d['value'],1), round(d['ms_per_step'],3), round(s['nmt_leaves']['avg_ms'],3))" >> $O/ab.txt
  done
done
unset CDA_LIB
cat $O/ab.txt
