#!/bin/bash
# A/B of x3s kernel variants (tools/build_x3s_variant.sh NAME ...): encoder stage times, interleaved, 2 passes.
# Usage on the box: bash tools/ab_x3s.sh default g1p1 g0p0 ...   ("default" = the in-tree library)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for pass in 1 2; do
  for v in "$@"; do
    if [ "$v" = default ]; then lib=$PWD/video-gen-evals_amd/vge/libvge.so; else lib=$PWD/video-gen-evals_amd/csrc/build/$v/libvge.so; fi
    VGE_LIB=$lib timeout -k 10 120 python -u tools/time_encoder.py --tag $v --calls 30 || exit $?
  done
done
