# r04zd: EDS-returned host pipeline vs batch size and host Q0-copy threads
set -e
mkdir -p gpurun_out/r04zd
cd $GRAFT_REPO_ROOT
for n in 256 512 1024; do
  for th in 8 2; do
    echo "n=$n CDA_HOST_THREADS=$th"
    CDA_HOST_THREADS=$th timeout -k 10 300 python tools/host_pipe_run.py $n 2 > gpurun_out/r04zd/n${n}_t${th}.log 2>&1 || { tail -5 gpurun_out/r04zd/n${n}_t${th}.log; exit 1; }
    grep "eds=True\|check" gpurun_out/r04zd/n${n}_t${th}.log
  done
done
