#!/bin/bash
# Local helper (never runs on the GPU box): submit one gpurun call, and when
# the pool has no free slot (gpurun exit code 3: nothing ran, nothing
# charged) submit it again after a pause.  Any other outcome -- success, a
# failure of the command itself, a refusal -- is returned as is: a failing GPU
# step is never retried.  Usage: tools/gpurun_wait.sh <timeout_s> '<command>'
T=$1; shift
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[gpurun_wait] no slot (attempt $i), retrying in 120 s"
  sleep 120
done
exit 3
