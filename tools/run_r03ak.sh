#!/bin/bash
# Round-3 GPU call "ak": whole trees per lane in the subtree launch where the
# levels run down to the roots (build_var/whole, -DCDA_SUBTREE_WHOLE=1: the
# subtree kernel writes the roots; config 4: 524288 lanes of 256-leaf trees)
# against the product (half trees + one level launch).
set -o pipefail
O=gpurun_out/r03ak
mkdir -p $O
B=$GRAFT_REPO_ROOT/celestia-app_amd/build_var
CDA_LIB=$B/whole/libcda.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_config4.py tests/test_gpu_parity.py -m gpu -k "all_1024 or multi_gpu or batch_of_32 or rank_shard" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for i in 1 2 3; do
  for v in prod whole; do
    if [ $v = whole ]; then export CDA_LIB=$B/whole/libcda.so; else unset CDA_LIB; fi
    timeout -k 10 200 python -u bench.py --no-cpu --no-extras --steps 10 --warmup 2 > $O/b.json 2>>$O/ab.err || exit 3
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); s=d['stages']; print('cfg4 $v', round(d['value'],1), round(d['ms_per_step'],3), round(s['nmt_levels']['avg_ms'],3), round(s['data_root']['avg_ms'],3))" >> $O/ab.txt
  done
done
unset CDA_LIB
cat $O/ab.txt
