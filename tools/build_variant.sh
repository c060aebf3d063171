#!/bin/bash
# Build a variant libvge.so with extra defines for vge_encoder_x3.hip into video-gen-evals_amd/csrc/build/<name>/
# (the rest from the in-tree objects).  Usage: tools/build_variant.sh NAME "-DVGE_TRACE -DFOO=1"
set -e
cd "$(dirname "$0")/../video-gen-evals_amd/csrc"
make -s ARCH=gfx950
mkdir -p build/$1
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 $2 -c vge_encoder_x3.hip -o build/$1/x3.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/$1/libvge.so build/vge_featurize.o build/vge_encoder.o \
  build/$1/x3.o build/vge_transformer_x3.o build/vge_score.o build/vge_api.o build/vge_ingest.o build/vge_vit.o \
  build/vge_cnn.o build/vge_pose_head.o build/vge_hmr.o build/vge_hmr_front.o build/vge_dwpose.o build/vge_yolox.o -lz -lpthread
