#!/bin/bash
# Round-3 GPU call "f" (run via gpurun from the repo root): GPU tests on the
# product library, the LDS_B variant's parity + latency A/B, the GF(2^8) slice
# mode A/B (CDA_RS8_SLICE=0/1, bench stage times), fixed-shape k = 128 PMC
# passes of the slice build, then the default bench line.  Every GPU step has
# its own time limit; the first failure ends the call.
set -o pipefail
O=gpurun_out/r03f
mkdir -p $O
V=$GRAFT_REPO_ROOT/celestia-app_amd/build_var/ldsb/libcda.so
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
CDA_LIB=$V timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k "512 or gf16" --timeout 120 --timeout-method thread > $O/ldsb_tests.log 2>&1 || { tail -30 $O/ldsb_tests.log; exit 2; }
for i in 1 2 3; do
  timeout -k 10 120 python -u tools/latency_ab.py >> $O/ldsb_ab.txt 2>>$O/ab.err || exit 3
  CDA_LIB=$V CDA_VARIANT=ldsb timeout -k 10 120 python -u tools/latency_ab.py >> $O/ldsb_ab.txt 2>>$O/ab.err || exit 3
done
for i in 1 2; do
  for S in 0 1; do
    CDA_RS8_SLICE=$S timeout -k 10 200 python -u bench.py --no-cpu --no-extras --steps 10 --warmup 2 > $O/slice${S}_$i.json 2>>$O/ab.err || exit 4
  done
done
echo "slice A/B done"
KS=128 timeout -k 10 900 tools/profile_round3.sh r03f || exit 5
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 6
tail -c 400 $O/bench.json
