# r04r: host pipeline D2H copy merging (CDA_D2H_MERGE 0/1/2) x copy-stream
# priority (CDA_COPY_PRIO 1/0), 1024 squares k=128, EDS returned; every
# variant's sampled EDS / data roots checked against the device path
set -e
mkdir -p gpurun_out/r04r
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for v in "CDA_D2H_MERGE=0 CDA_COPY_PRIO=0" "CDA_D2H_MERGE=0 CDA_COPY_PRIO=1" "CDA_D2H_MERGE=1 CDA_COPY_PRIO=1" "CDA_D2H_MERGE=2 CDA_COPY_PRIO=1"; do
    echo "[$v] $(env $v timeout -k 10 300 python tools/host_pipe_run.py 1024 2 2>&1 | grep 'eds=True\|check' | tr '\n' ' ')"
  done
done
