# r04zg: EDS-returned host pipeline (streaming-store Q0 copy) vs host copy threads
set -e
mkdir -p gpurun_out/r04zg
cd $GRAFT_REPO_ROOT
for pass in 1 2; do
  for th in 4 8 12; do
    echo "pass $pass CDA_HOST_THREADS=$th"
    CDA_HOST_THREADS=$th timeout -k 10 300 python tools/host_pipe_run.py 1024 2 > gpurun_out/r04zg/p${pass}_t${th}.log 2>&1 || { tail -5 gpurun_out/r04zg/p${pass}_t${th}.log; exit 1; }
    grep "eds=True\|check" gpurun_out/r04zg/p${pass}_t${th}.log
  done
done
