#!/bin/bash
# Round-3 GPU call "al": the final round-3 build (k-dependent subtree lane target) --
# GPU suite, smoke(), fixed-shape traces + PMC passes (profile tag r03zzd),
# then the default bench line against that summary (copied into profiles/
# first so bench.py reads it).
set -o pipefail
O=gpurun_out/r03av
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
KS="128 512" timeout -k 10 900 tools/profile_round3.sh r03zzd > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 3; }
tail -1 $O/profile.log
cd $R && cp gpurun_out/r03zzd_pmc.json profiles/ || exit 4
for i in 1 2; do
  timeout -k 10 400 python -u bench.py > $O/bench_$i.json 2> $O/bench_$i.err || { tail -20 $O/bench_$i.err; exit 5; }
  python3 -c "import json; d=json.loads(open('$O/bench_$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['extras']['latency_single_square_ms'], d['extras']['k512']['ms_per_square'])"
done
