# r04s: round-4 evidence -- fixed-shape kernel trace + PMC passes (k=128 config-4
# batch, k=512 one square) of the product build, then the full default bench
set -e
cd $GRAFT_REPO_ROOT
KS="128 512" bash tools/profile_round3.sh r04s
timeout -k 10 900 python bench.py > gpurun_out/r04s_bench.log 2>&1
tail -c 600 gpurun_out/r04s_bench.log
