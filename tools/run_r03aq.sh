#!/bin/bash
# Round-3 GPU call "aq": subtree_kernel without the one-node-ahead prefetch
# (operands loaded at use): 141 VGPRs = three waves per SIMD (build_var/nopf3)
# or held to 128 = four (build_var/nopf4, 9 spills), against the product
# (189 VGPRs, two waves), at subtree lane targets 131072 / 262144:
# 128- and 1024-square k=128 batches, one k=512 square.
set -o pipefail
O=gpurun_out/r03aq
mkdir -p $O
B=$GRAFT_REPO_ROOT/celestia-app_amd/build_var
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
for v in nopf3 nopf4; do
  CDA_LIB=$B/$v/libcda.so CDA_SUBTREE_LANES=262144 timeout -k 10 300 $T tests/test_config4.py tests/test_gpu_parity.py -m gpu -k "all_1024 or rank_shard or batch_of_32 or k512" >> $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
done
grep -E "passed|failed" $O/parity.log
for i in 1 2; do
  for v in prod nopf3 nopf4; do
    for L in 131072 262144; do
      if [ $v = prod ]; then unset CDA_LIB; else export CDA_LIB=$B/$v/libcda.so; fi
      export CDA_SUBTREE_LANES=$L CDA_VARIANT=$v
      for n in 128 1024; do
        timeout -k 10 200 python -u bench.py --batch $n --distinct 16 --no-cpu --no-extras --steps 10 --warmup 2 > $O/b.json 2>>$O/ab.err || exit 3
        python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); s=d['stages']; print('n=$n $v $L', round(d['value'],1), round(d['ms_per_step'],4), round(s['nmt_levels']['avg_ms'],4))" >> $O/ab.txt
      done
      if [ $i = 1 ]; then timeout -k 10 120 python -u tools/latency_ab.py >> $O/lat.txt 2>>$O/ab.err || exit 2; fi
    done
  done
done
unset CDA_LIB CDA_SUBTREE_LANES CDA_VARIANT
cat $O/ab.txt
python3 -c "
import json
for l in open('$O/lat.txt'):
    d=json.loads(l); e=d['env']; print(e.get('CDA_VARIANT'), e.get('CDA_SUBTREE_LANES'), round(d['k128_ms_median'],4), round(d['k512_ms_median'],4), round(d['k512_ms_min'],4))
"
