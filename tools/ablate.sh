#!/bin/bash
# Build timing-only variants of the 3xfp16 encoder + transformer kernels into video-gen-evals_amd/csrc/build/:
#   ablN/libvge.so  for each VGE_ABL bit mask N given as an argument (see vge_x3.h; transformer: 32 L2-resident
#                   weights, 64 no CLS dot products, 128 no stream barriers)
#   trace/libvge.so with VGE_TRACE (s_memtime phase stamps, read by tools/trace_encoder.py)
# Run them on the GPU box with VGE_LIB=<that path> python tools/time_encoder.py / trace_encoder.py.
set -e
cd "$(dirname "$0")/../video-gen-evals_amd/csrc"
make -s ARCH=gfx950
HIPCC="/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950"
link() {
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$1/libvge.so" "${FEAT:-build/vge_featurize.o}" \
    build/vge_encoder.o "$1/x3.o" "$1/tx.o" build/vge_score.o build/vge_api.o build/vge_ingest.o build/vge_vit.o \
    build/vge_cnn.o build/vge_pose_head.o build/vge_hmr.o build/vge_hmr_front.o build/vge_dwpose.o build/vge_yolox.o -lz -lpthread
}
for v in "$@"; do
  mkdir -p build/abl$v
  $HIPCC -DVGE_ABL=$v -c vge_encoder_x3.hip -o build/abl$v/x3.o
  $HIPCC -DVGE_ABL=$v -c vge_transformer_x3.hip -o build/abl$v/tx.o
  $HIPCC -DVGE_ABL=$v -c vge_featurize.hip -o build/abl$v/feat.o
  FEAT=build/abl$v/feat.o link build/abl$v
done
mkdir -p build/trace
$HIPCC -DVGE_TRACE -c vge_encoder_x3.hip -o build/trace/x3.o
$HIPCC -DVGE_TRACE -c vge_transformer_x3.hip -o build/trace/tx.o
link build/trace
mkdir -p build/trace2  # conv stamps of round 2 (the pair units at 256 windows)
$HIPCC -DVGE_TRACE -DVGE_TRACE_ROUND=2 -c vge_encoder_x3.hip -o build/trace2/x3.o
cp build/trace/tx.o build/trace2/tx.o
link build/trace2
