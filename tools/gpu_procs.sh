#!/bin/bash
# Count the processes that hold a GPU device node open (/dev/kfd or a DRM
# render node) while a command runs: samples every second, prints the largest
# sample with each process's command line.  Usage: bash tools/gpu_procs.sh <cmd...>
"$@" &
P=$!
best=0
while kill -0 $P 2>/dev/null; do
  cur=()
  for d in /proc/[0-9]*; do
    if ls -l $d/fd 2>/dev/null | grep -qE '/dev/kfd|/dev/dri/render'; then
      cur+=("${d#/proc/} $(tr '\0' ' ' < $d/cmdline 2>/dev/null | cut -c1-150)")
    fi
  done
  if [ ${#cur[@]} -gt $best ]; then best=${#cur[@]}; snap=("${cur[@]}"); fi
  sleep 1
done
wait $P; rc=$?
echo "max processes with a GPU node open: $best"
printf '%s\n' "${snap[@]}"
exit $rc
