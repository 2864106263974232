#!/bin/bash
# Round-3 GPU call "i": the GPU suite (with the variant tests), then kernel
# timelines of one k = 128 and one k = 512 square (config 2 / config 3
# latency chains) from rocprofv3 kernel traces.
set -o pipefail
O=gpurun_out/r03i
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
cd /tmp && export TMPDIR=/tmp
for K in 128 512; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/lat$K -o run -- python3 $R/tools/latency_profile.py $K > $R/$O/lat$K.log 2>&1 || exit 2
  python3 $R/tools/trace_timeline.py $R/$O/lat$K 12 > $R/$O/k${K}_timeline.txt || exit 3
  cat $R/$O/k${K}_timeline.txt
done
