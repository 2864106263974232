#!/bin/bash
# Builds timeline variants of libcda.so (rs_gf16.hip with CDA_RS16_TRACE=1, 2)
# into tools/var/rs16_trace<N>/libcda.so; outputs stay bit-exact (the trace
# only adds clock reads and one store per phase from one lane).  GPU side:
# python tools/rs16_trace.py tools/var/rs16_trace1/libcda.so
set -e
cd "$(dirname "$0")/../celestia-app_amd"
make -s libcda.so
OBJS=$(ls build/*.o | grep -v rs_gf16.o)
for p in ${VARIANTS:-1 2}; do
  out=../tools/var/rs16_trace$p
  mkdir -p $out
  /opt/rocm/bin/hipcc -O3 -std=c++20 -fPIC --offload-arch=gfx950 -DCDA_RS16_TRACE=$p $EXTRA -c csrc/rs_gf16.hip -o $out/rs_gf16.o
  /opt/rocm/bin/hipcc -O3 -std=c++20 -fPIC --offload-arch=gfx950 -shared -o $out/libcda.so $out/rs_gf16.o $OBJS \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  rm $out/rs_gf16.o
done
