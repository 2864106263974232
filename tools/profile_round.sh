#!/bin/bash
# A round's evidence in one GPU call: the GPU suite, smoke() and the default
# bench (tools/run_round.sh), then the fixed-shape kernel traces + PMC passes
# of tools/profile_round3.sh (k = 128: config 4's 1024 squares per step;
# k = 512: one square per step).  Usage: bash tools/profile_round.sh <tag>
set -o pipefail
TAG=${1:?tag}
bash tools/run_round.sh "$TAG" || exit $?
bash tools/profile_round3.sh "$TAG" > "gpurun_out/$TAG/profile.log" 2>&1
