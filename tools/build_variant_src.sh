#!/bin/bash
# Build a variant libvge.so with extra defines for ONE source file into video-gen-evals_amd/csrc/build/<name>/ (the
# rest from the in-tree objects).  Usage: tools/build_variant_src.sh NAME SOURCE.hip "-DVGE_ABL=64 ..."
set -e
cd "$(dirname "$0")/../video-gen-evals_amd/csrc"
make -s ARCH=gfx950
mkdir -p build/$1
src=$2; base=${src%.hip}
extra=""; [ "$base" = vge_encoder_x3s ] && extra="-fno-slp-vectorize"
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 $extra $3 -c $src -o build/$1/$base.o
objs=$(ls build/*.o | grep -v "build/$base.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/$1/libvge.so $objs build/$1/$base.o -L/opt/rocm/lib -lhipblaslt -Wl,-rpath,/opt/rocm/lib -lz -lpthread
