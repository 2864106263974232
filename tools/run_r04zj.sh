# r04zj: EDS-returned host pipeline, host Q0 copy paced after the enqueue loop by per-chunk D2H events (CDA_HOST_Q0_PACED) vs one burst
set -e
mkdir -p gpurun_out/r04zj
cd $GRAFT_REPO_ROOT
for pass in 1 2 3; do
  for p in 1 0; do
    echo "pass $pass CDA_HOST_Q0_PACED=$p"
    CDA_HOST_Q0_PACED=$p timeout -k 10 300 python tools/host_pipe_run.py 1024 2 > gpurun_out/r04zj/p${pass}_q${p}.log 2>&1 || { tail -5 gpurun_out/r04zj/p${pass}_q${p}.log; exit 1; }
    grep "eds=True\|check" gpurun_out/r04zj/p${pass}_q${p}.log
  done
done
