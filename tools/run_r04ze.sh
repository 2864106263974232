# r04ze: EDS-returned host pipeline, Q0 host copy with streaming stores (CDA_HOST_NT) x threads
set -e
mkdir -p gpurun_out/r04ze
cd $GRAFT_REPO_ROOT
for pass in 1 2; do
for nt in 1 0; do
  for th in 8 16; do
    echo "pass $pass n=1024 CDA_HOST_NT=$nt CDA_HOST_THREADS=$th"
    CDA_HOST_NT=$nt CDA_HOST_THREADS=$th timeout -k 10 300 python tools/host_pipe_run.py 1024 2 > gpurun_out/r04ze/p${pass}_nt${nt}_t${th}.log 2>&1 || { tail -5 gpurun_out/r04ze/p${pass}_nt${nt}_t${th}.log; exit 1; }
    grep "eds=True\|check" gpurun_out/r04ze/p${pass}_nt${nt}_t${th}.log
  done
done
done
