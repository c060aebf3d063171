#!/bin/bash
# Build timing-only ablation variants of the 3xfp16 encoder kernels (VGE_ABL bit masks given as arguments,
# see vge_encoder_x3.hip) into video-gen-evals_amd/csrc/build/ablN/libvge.so.  Run them on the GPU box with:
#   for v in MASKS; do VGE_LIB=... python tools/time_encoder.py --tag abl$v; done
set -e
cd "$(dirname "$0")/../video-gen-evals_amd/csrc"
make -s ARCH=gfx950
for v in "$@"; do
  mkdir -p build/abl$v
  /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -DVGE_ABL=$v -c vge_encoder_x3.hip -o build/abl$v/x3.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/abl$v/libvge.so build/vge_featurize.o \
    build/vge_encoder.o build/abl$v/x3.o build/vge_score.o build/vge_api.o
done
