#!/bin/bash
# Round-3 GPU call "n": data-root pad-row prefetch (early request, LDS-only
# phase barriers) -- parity, latency A/B against -DCDA_DR_LATE_PAD, and the
# phase trace of both.
set -o pipefail
O=gpurun_out/r03n
mkdir -p $O
B=$GRAFT_REPO_ROOT/celestia-app_amd/build_var
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py tests/test_dah.py tests/test_config4.py -m gpu -k "not all_1024 and not multi_gpu" > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for i in 1 2 3; do
  CDA_LIB=$B/latepad/libcda.so CDA_VARIANT=latepad timeout -k 10 120 python -u tools/latency_ab.py >> $O/pad_ab.txt 2>>$O/ab.err || exit 2
  timeout -k 10 120 python -u tools/latency_ab.py >> $O/pad_ab.txt 2>>$O/ab.err || exit 2
done
cat $O/pad_ab.txt
CDA_LIB=$B/toptrace/libcda.so timeout -k 10 120 python -u tools/top_trace.py > $O/trace_new.txt 2>>$O/ab.err || exit 3
CDA_LIB=$B/toptrace_late/libcda.so timeout -k 10 120 python -u tools/top_trace.py > $O/trace_late.txt 2>>$O/ab.err || exit 3
paste $O/trace_late.txt $O/trace_new.txt
