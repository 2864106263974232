#!/bin/bash
# Round-3 GPU call "ac": the build with subtree levels down to the roots --
# GPU suite, smoke(), fixed-shape traces + PMC passes (tools/profile_round3.sh),
# then the default bench line (which reads the newest profiles/*_pmc.json:
# copy gpurun_out/r03ac_pmc.json to profiles/ and re-run the bench for the
# committed line).
set -o pipefail
O=gpurun_out/r03ac
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
KS="128 512" timeout -k 10 900 tools/profile_round3.sh r03ac > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 3; }
tail -1 $O/profile.log
