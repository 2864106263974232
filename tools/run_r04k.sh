# r04k: host pipeline (config 4 from pinned host buffers, EDS returned):
# memory-copy + kernel trace of one 256-square call, and the copy-shape A/B
# (full EDS D2H vs Q1 2-D + Q2|Q3 linear)
set -e
mkdir -p gpurun_out/r04k
cd $GRAFT_REPO_ROOT
for v in 0 1; do echo "full_d2h=$v"; CDA_HOST_FULL_D2H=$v timeout -k 10 200 python tools/host_pipe_run.py 512 2 2>&1 | grep eds=True; done > gpurun_out/r04k/shape.txt 2>&1
cat gpurun_out/r04k/shape.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04k/prof -o pipe -- python3 $GRAFT_REPO_ROOT/tools/host_pipe_run.py 256 1 > $GRAFT_REPO_ROOT/gpurun_out/r04k/prof.log 2>&1
ls $GRAFT_REPO_ROOT/gpurun_out/r04k/prof
