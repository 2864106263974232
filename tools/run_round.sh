#!/bin/bash
# GPU-box script (gpurun): the GPU suite, smoke() and the default bench, each
# under its own time limit, stopping at the first failure.  Output under
# gpurun_out/<tag>/.  Usage: bash tools/run_round.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:?tag}
K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
ARGS=(tests -m gpu -x -v --timeout 300 --timeout-method thread)
[ -n "$K" ] && ARGS+=(-k "$K")
timeout -k 10 900 python -u -m pytest "${ARGS[@]}" > "$OUT/gpu_tests.log" 2>&1 || exit $?
[ -n "$K" ] && exit 0
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > "$OUT/bench.log" 2>&1
