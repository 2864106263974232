#!/bin/bash
# Builds timing-diagnostic variants of libcda.so that differ only in
# rs_gf8_bs.hip's CDA_RS8_PROBE (1 = no compute, 2 = no global memory,
# 3 = no LDS exchange, 4 = RS a no-op) into tools/var/probe<N>/libcda.so.  Their output is
# wrong by construction: run bench.py with CDA_LIB=<variant> and
# CDA_BENCH_NOCHECK=1 and read only the rs_q0 / rs_q3 stage times.
set -e
cd "$(dirname "$0")/../celestia-app_amd"
make -s libcda.so
OBJS=$(ls build/*.o | grep -v rs_gf8_bs.o)
for p in 1 2 3 4; do
  out=../tools/var/probe$p
  mkdir -p $out
  /opt/rocm/bin/hipcc -O3 -std=c++20 -fPIC --offload-arch=gfx950 -DCDA_RS8_PROBE=$p -c csrc/rs_gf8_bs.hip -o $out/rs_gf8_bs.o
  /opt/rocm/bin/hipcc -O3 -std=c++20 -fPIC --offload-arch=gfx950 -shared -o $out/libcda.so $out/rs_gf8_bs.o $OBJS \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  rm $out/rs_gf8_bs.o
done
