#!/bin/bash
# Builds timing-diagnostic variants of libcda.so that differ only in
# rs_gf16.hip's CDA_RS16_PROBE (1 = no butterflies, 2 = no global memory) into
# tools/var/rs16_probe<N>/libcda.so (wrong output by construction).  GPU side:
# for v in 1 2; do CDA_LIB=$PWD/tools/var/rs16_probe$v/libcda.so CDA_BENCH_NOCHECK=1 python bench.py --k 512 ...
set -e
cd "$(dirname "$0")/../celestia-app_amd"
make -s libcda.so
OBJS=$(ls build/*.o | grep -v rs_gf16.o)
for p in 1 2; do
  out=../tools/var/rs16_probe$p
  mkdir -p $out
  /opt/rocm/bin/hipcc -O3 -std=c++20 -fPIC --offload-arch=gfx950 -DCDA_RS16_PROBE=$p -c csrc/rs_gf16.hip -o $out/rs_gf16.o
  /opt/rocm/bin/hipcc -O3 -std=c++20 -fPIC --offload-arch=gfx950 -shared -o $out/libcda.so $out/rs_gf16.o $OBJS \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  rm $out/rs_gf16.o
done
