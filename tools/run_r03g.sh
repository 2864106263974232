#!/bin/bash
# Round-3 GPU call "g" (run via gpurun from the repo root): parity of the
# half-width GF(2^16) kernel (product default), the GPU suite, latency A/B of
# CDA_RS16_HALF=0/1 and of the pass-B LDS variant, the GF(2^8) slice-mode A/B
# (CDA_RS8_SLICE=0/1, bench stage times).  Every GPU step has its own time
# limit; the first failure ends the call.
set -o pipefail
O=gpurun_out/r03g
mkdir -p $O
V=$GRAFT_REPO_ROOT/celestia-app_amd/build_var/ldsb/libcda.so
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 200 $T tests/test_gpu_parity.py -m gpu -k "512 or 256 or gf16" > $O/half_parity.log 2>&1 || { tail -30 $O/half_parity.log; exit 1; }
tail -1 $O/half_parity.log
timeout -k 10 400 $T tests -m gpu > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 2; }
tail -1 $O/gpu_tests.log
CDA_LIB=$V timeout -k 10 200 $T tests/test_gpu_parity.py -m gpu -k "512 or 256 or gf16" > $O/ldsb_tests.log 2>&1 || { tail -30 $O/ldsb_tests.log; exit 3; }
for i in 1 2 3; do
  CDA_RS16_HALF=0 timeout -k 10 120 python -u tools/latency_ab.py >> $O/half_ab.txt 2>>$O/ab.err || exit 4
  timeout -k 10 120 python -u tools/latency_ab.py >> $O/half_ab.txt 2>>$O/ab.err || exit 4
  CDA_LIB=$V CDA_VARIANT=ldsb timeout -k 10 120 python -u tools/latency_ab.py >> $O/half_ab.txt 2>>$O/ab.err || exit 4
done
cat $O/half_ab.txt
for i in 1 2; do
  for S in 0 1; do
    CDA_RS8_SLICE=$S timeout -k 10 200 python -u bench.py --no-cpu --no-extras --steps 10 --warmup 2 > $O/slice${S}_$i.json 2>>$O/ab.err || exit 5
  done
done
echo "slice A/B done"
