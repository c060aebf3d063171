#!/bin/bash
# Build a variant libvge.so with extra defines for vge_encoder_x3s.hip into video-gen-evals_amd/csrc/build/<name>/
# (the rest from the in-tree objects).  Usage: tools/build_x3s_variant.sh NAME "-DVGE_TRACE -DFOO=1"
set -e
cd "$(dirname "$0")/../video-gen-evals_amd/csrc"
make -s ARCH=gfx950
mkdir -p build/$1
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -fno-slp-vectorize $2 -c vge_encoder_x3s.hip -o build/$1/x3s.o
objs=$(ls build/*.o | grep -v vge_encoder_x3s.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/$1/libvge.so $objs build/$1/x3s.o -lz -lpthread
