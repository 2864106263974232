#!/bin/bash
# Round-3 GPU call "o": fixed-shape kernel traces + PMC passes of the build
# with the LDS-DMA GF(2^16) staging and the fused subtree levels
# (tools/profile_round3.sh), then the default bench line.
set -o pipefail
O=gpurun_out/r03o
mkdir -p $O
KS="128 512" timeout -k 10 900 tools/profile_round3.sh r03o > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
tail -1 $O/profile.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 2; }
tail -c 600 $O/bench.json
