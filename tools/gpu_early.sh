#!/bin/bash
# first-conv epilogues exchanging a bound of their maxima before the GELUs (build/early) vs the in-tree kernel
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in default early; do
  if [ "$v" = default ]; then lib=$PWD/video-gen-evals_amd/vge/libvge.so; else lib=$PWD/video-gen-evals_amd/csrc/build/$v/libvge.so; fi
  VGE_LIB=$lib timeout -k 10 120 python -u tools/enc_dump.py gpurun_out/dump_$v.npz || exit $?
done
python tools/enc_compare.py gpurun_out/dump_default.npz gpurun_out/dump_early.npz
bash tools/ab_x3s.sh default early 2>&1 | grep tag || exit 1
bash tools/ab_x3s.sh default early 2>&1 | grep tag || exit 1
