#!/bin/bash
# Build libvge variants with GEMM ablation bits (VGE_GABL) into tools/abl/ (timing only: wrong results).
set -e
cd "$(dirname "$0")/../video-gen-evals_amd/csrc"
mkdir -p ../../tools/abl build/abl
OBJS=$(ls build/*.o | grep -v vge_vit.o)
for A in "$@"; do
  /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -DVGE_GABL=$A -c vge_vit.hip -o build/abl/vit_$A.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/abl/libvge_gabl$A.so $OBJS build/abl/vit_$A.o -lz -lpthread
done
