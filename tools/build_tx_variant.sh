#!/bin/bash
# Build a variant libvge.so with extra defines for vge_transformer_x3.hip into video-gen-evals_amd/csrc/build/<name>/
# (the rest from the in-tree objects).  Usage: tools/build_tx_variant.sh NAME "-DVGE_ABL=64"
set -e
cd "$(dirname "$0")/../video-gen-evals_amd/csrc"
make -s ARCH=gfx950
mkdir -p build/$1
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 $2 -c vge_transformer_x3.hip -o build/$1/tx.o
objs=$(ls build/*.o | grep -v vge_transformer_x3.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/$1/libvge.so $objs build/$1/tx.o -lz -lpthread
