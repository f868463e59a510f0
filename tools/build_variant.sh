#!/bin/bash
# Experiment build of libaqchip: mps.hip (the two-site chain and the Gram SVD) recompiled with extra
# -D flags, linked with the default build's other objects into adaptaqc_amd/libaqchip_<tag>.so
# (selected at run time by AQC_LIB, tools/ab_repeat.sh).  Run here (CPU), after `make`.
# Usage: bash tools/build_variant.sh <tag> -DNAME=VALUE ...
set -e
tag=$1; shift
cd "$(dirname "$0")/../adaptaqc_amd/csrc"
make -s
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -Wno-unused-value \
  -munsafe-fp-atomics "$@" -c mps.hip -o build/mps_$tag.o
objs=$(ls build/*.o | grep -v "build/mps" | tr '\n' ' ')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../libaqchip_$tag.so $objs build/mps_$tag.o \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built adaptaqc_amd/libaqchip_$tag.so"
