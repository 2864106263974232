#!/bin/bash
# Fused encode + leaves vs separate launches (k = 128, 128 squares per step):
# kernel trace, then instruction-fetch and issue counters in separate --pmc
# passes, for CDA_RS8_FUSED=0 and =1 on the test build.  Usage: tools/fused_pmc.sh TAG
set -e
TAG=${1:?tag}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --batch 128 --no-cpu --no-extras --steps 3 --warmup 1"
export CDA_LIB=$GRAFT_REPO_ROOT/celestia-app_amd/libcda_test.so
for F in 0 1; do
  export CDA_RS8_FUSED=$F
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace$F -o run -- python3 $B > $OUT/trace$F.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --output-format csv -d $OUT/ic$F -o run -- python3 $B > $OUT/ic$F.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq$F -o run -- python3 $B > $OUT/sq$F.log 2>&1
done
