#!/bin/bash
# Round-3 GPU call "ah": kernel timelines of one k = 128 and one k = 512 square
# on the final build (rocprofv3 kernel trace, tools/trace_timeline.py).
set -o pipefail
O=gpurun_out/r03ah
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for K in 128 512; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/lat$K -o run -- python3 $R/tools/latency_profile.py $K > $R/$O/lat$K.log 2>&1 || exit 2
  python3 $R/tools/trace_timeline.py $R/$O/lat$K 14 > $R/$O/k${K}_timeline.txt || exit 3
  cat $R/$O/k${K}_timeline.txt
done
