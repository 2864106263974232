#!/bin/bash
# Instruction-fetch counters per kernel for the k = 512 path (run via gpurun):
# SQC_ICACHE_* in one pass, SQ_IFETCH / SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES /
# SQ_WAIT_ANY / SQ_BUSY_CYCLES in another.  Summary: tools/icache_summary.py.
set -e
OUT=${OUT:-$GRAFT_REPO_ROOT/gpurun_out/icache}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --k 512 --batch 4 --no-cpu --no-extras --steps 3 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --output-format csv -d $OUT/ic -o run -- python3 $B > $OUT/ic.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/sq -o run -- python3 $B > $OUT/sq.log 2>&1
