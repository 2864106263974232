#!/bin/bash
# Round-3 GPU call "z": memory-only replicas of the k = 128 Q0 RS launch
# (tools/rs8_pattern_probe) beside the product's Q0 stage time.
set -o pipefail
O=gpurun_out/r03z
mkdir -p $O
timeout -k 10 200 ./tools/rs8_pattern_probe 1024 > $O/pattern.txt 2>&1 || { cat $O/pattern.txt; exit 1; }
cat $O/pattern.txt
