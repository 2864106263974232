#!/bin/bash
# Build a variant of libcda.so with extra compile flags (A/B experiments):
#   tools/build_variant.sh <name> <flags...>  ->  celestia-app_amd/build_var/<name>/libcda.so
# Load it with CDA_LIB=<path> (celestia_da/_lib.py); the product library is
# untouched.
set -e
NAME=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/celestia-app_amd/build_var/$NAME
mkdir -p $OUT/obj
make -C $R/celestia-app_amd -j8 BUILD=$OUT/obj LIB=$OUT/libcda.so HIPFLAGS="-O3 -std=c++20 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $*" >/dev/null
rm -rf $OUT/obj   # objects stay local: only the library travels to the GPU box
echo $OUT/libcda.so
