#!/bin/bash
# Round-3 GPU call "aa": fused subtree levels for config 4's 1024-square batch
# (build_var/st1, -DCDA_SUBTREE_STOP1=1: subtrees also where the per-level
# launches run down to the roots; CDA_SUBTREE_LANES picks the subtree size:
# 131072 -> 128-leaf subtrees, 2^21 -> 64, 2^23 -> 16) against the product.
set -o pipefail
O=gpurun_out/r03aa
mkdir -p $O
B=$GRAFT_REPO_ROOT/celestia-app_amd/build_var
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
for L in 131072 2097152 8388608; do
  CDA_LIB=$B/st1/libcda.so CDA_SUBTREE_LANES=$L timeout -k 10 200 $T tests/test_config4.py -m gpu -k "all_1024" >> $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
done
grep -E "passed|failed" $O/parity.log
for i in 1 2; do
  for v in prod 131072 2097152 8388608; do
    if [ $v = prod ]; then unset CDA_LIB CDA_SUBTREE_LANES; else export CDA_LIB=$B/st1/libcda.so CDA_SUBTREE_LANES=$v; fi
    timeout -k 10 200 python -u bench.py --no-cpu --no-extras --steps 10 --warmup 2 > $O/b_${v}_$i.json 2>>$O/ab.err || exit 3
    python3 -c "import json; d=json.loads(open('$O/b_${v}_$i.json').read().strip().splitlines()[-1]); s=d['stages']; print('cfg4 $v', round(d['value'],1), round(d['ms_per_step'],3), *[(k, round(s[k]['avg_ms'],3)) for k in ('nmt_leaves','nmt_levels','data_root')])" >> $O/ab.txt
  done
done
unset CDA_LIB CDA_SUBTREE_LANES
cat $O/ab.txt
