set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/k512
mkdir -p $OUT
cd /tmp; export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --k 512 --batch 1 --distinct 1 --no-cpu --no-extras --steps 4 --warmup 1"
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $B > $OUT/trace.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS --output-format csv -d $OUT/sq -o run -- python3 $B > $OUT/sq.log 2>&1 || exit 2
echo done
