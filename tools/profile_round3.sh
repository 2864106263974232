#!/bin/bash
# Round-3 evidence in one GPU call (run via gpurun), fixed launch shapes so
# every per-launch counter divides by a known square count:
#   k = 128: config 4's 1024 squares per step (bench default: one hash stream)
#   k = 512: one square per step (config 3)
# kernel trace + stats, then separate --pmc passes (FETCH_SIZE; WRITE_SIZE; SQ
# issue counters; SQ wait counters), summarised by tools/pmc_summary3.py into
# gpurun_out/<tag>_pmc.json.  Usage: [KS="128"] tools/profile_round3.sh <tag>
set -o pipefail
TAG=${1:-r03}
R=$GRAFT_REPO_ROOT
cd /tmp
export TMPDIR=/tmp

SUM=$R/gpurun_out/${TAG}_pmc.json
rm -f $SUM
for K in ${KS:-128 512}; do
  OUT=$R/gpurun_out/prof_${TAG}_k$K
  rm -rf $OUT; mkdir -p $OUT
  if [ $K = 128 ]; then
    B="$R/bench.py --no-cpu --no-extras --steps 3 --warmup 1"; STEPS=7; SQ=1024
  else
    B="$R/bench.py --k 512 --batch 1 --distinct 1 --no-cpu --no-extras --steps 4 --warmup 1"; STEPS=9; SQ=1
  fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.log 2>&1 || exit 1
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $B > $OUT/fetch.log 2>&1 || exit 2
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $B > $OUT/write.log 2>&1 || exit 3
  timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- python3 $B > $OUT/sq.log 2>&1 || exit 4
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/wait -o run -- python3 $B > $OUT/wait.log 2>&1 || exit 5
  cd $R && python3 tools/pmc_summary3.py $OUT $SUM $K $STEPS $SQ "python3 ${B#$R/}" > $OUT/pmc_summary.log 2>&1 || exit 6
  cp $OUT/trace/run_kernel_stats.csv $R/gpurun_out/${TAG}_k${K}_kernel_stats.csv
  cd /tmp
done
echo profile done
