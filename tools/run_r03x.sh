#!/bin/bash
# Round-3 GPU call "x": HBM bandwidth by read : write mix (tools/bw_probe).
set -o pipefail
O=gpurun_out/r03x
mkdir -p $O
timeout -k 10 120 ./tools/bw_probe > $O/bw_probe.txt 2>&1 || { cat $O/bw_probe.txt; exit 1; }
cat $O/bw_probe.txt
