#!/bin/bash
# rs16_cw_kernel<512> stall counters (round-3 evidence for DESIGN 3.4 / 7.1):
# three separate rocprofv3 --pmc passes over one-square k=512 bench runs.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/rs16_stall
mkdir -p $OUT
cd /tmp
export TMPDIR=/tmp
B="$R/bench.py --k 512 --batch 1 --distinct 1 --no-cpu --no-extras --steps 4 --warmup 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SMEM SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/a -o run -- python3 $B > $OUT/a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_INST_LEVEL_SMEM SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $OUT/b -o run -- python3 $B > $OUT/b.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVES SQ_IFETCH SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR --output-format csv -d $OUT/c -o run -- python3 $B > $OUT/c.log 2>&1 || exit 3
echo done
