#!/bin/bash
# Build a variant of libcda.so with extra compile flags (A/B experiments):
#   tools/build_variant.sh <name> <flags...>  ->  celestia-app_amd/build_var/<name>/libcda.so
# PATCH=<file> (e.g. tools/probes/rs16_phases.patch) builds from a scratch
# copy of the package with that patch applied, so timing probes never live in
# the product source.  Load the result with CDA_LIB=<path>
# (celestia_da/_lib.py); the product library is untouched.
set -e
NAME=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/celestia-app_amd/build_var/$NAME
mkdir -p $OUT/obj
PKG=$R/celestia-app_amd
if [ -n "$PATCH" ]; then
  T=$(mktemp -d)
  mkdir -p $T/include $T/pkg
  cp $R/include/cda.h $T/include/
  cp -r $PKG/csrc $PKG/Makefile $T/pkg/
  patch -s -d $T/pkg -p1 < "$PATCH"
  PKG=$T/pkg
fi
# -DCDA_TESTING: a variant is a test build, so the A/B knobs (csrc/knobs.h) still apply to it
make -C $PKG -j8 BUILD=$OUT/obj LIB=$OUT/libcda.so HIPFLAGS="-O3 -std=c++20 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -DCDA_TESTING $*" >/dev/null
rm -rf $OUT/obj   # objects stay local: only the library travels to the GPU box
[ -n "$PATCH" ] && rm -rf "$T"
echo $OUT/libcda.so
