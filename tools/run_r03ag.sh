#!/bin/bash
# Round-3 GPU call "ag": does the leaf kernel's HBM traffic cost it clock?
# build_var/alias (-DCDA_LEAF_ALIAS_PROBE, wrong output: every square's leaves
# read square 0's cells, so the EDS reads hit L2 / MALL) against the product,
# config 4 stage times, plus the leaf kernel's clock from one SQ/GRBM pass each.
set -o pipefail
O=gpurun_out/r03ag
mkdir -p $O
B=$GRAFT_REPO_ROOT/celestia-app_amd/build_var
for i in 1 2; do
  for v in prod alias; do
    if [ $v = alias ]; then export CDA_LIB=$B/alias/libcda.so CDA_BENCH_NOCHECK=1; else unset CDA_LIB CDA_BENCH_NOCHECK; fi
    timeout -k 10 200 python -u bench.py --no-cpu --no-extras --steps 10 --warmup 2 > $O/b.json 2>>$O/ab.err || exit 3
    python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); s=d['stages']; print('cfg4 $v', round(d['value'],1), round(d['ms_per_step'],3), round(s['nmt_leaves']['avg_ms'],3), round(s['nmt_levels']['avg_ms'],3))" >> $O/ab.txt
  done
done
cat $O/ab.txt
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in prod alias; do
  if [ $v = alias ]; then export CDA_LIB=$B/alias/libcda.so CDA_BENCH_NOCHECK=1; else unset CDA_LIB CDA_BENCH_NOCHECK; fi
  timeout -s KILL 200 rocprofv3 --pmc SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU --output-format csv -d $R/$O/pmc_$v -o run -- python3 $R/bench.py --no-cpu --no-extras --steps 2 --warmup 1 > $R/$O/pmc_$v.log 2>&1 || exit 4
done
echo pmc done
