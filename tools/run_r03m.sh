#!/bin/bash
# Round-3 GPU call "m": the GPU suite (with config 4's N = 2 / N = 4 per-GPU
# shard tests), then the tree-top / data-root phase trace (CDA_TOP_TRACE
# variant) for configs 2 and 3.
set -o pipefail
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
CDA_LIB=$GRAFT_REPO_ROOT/celestia-app_amd/build_var/toptrace/libcda.so timeout -k 10 120 python -u tools/top_trace.py > $O/top_trace.txt 2>$O/top_trace.err || { tail -20 $O/top_trace.err; exit 2; }
cat $O/top_trace.txt
