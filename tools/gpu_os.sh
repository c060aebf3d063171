#!/bin/bash
# conv chain as one (GEMM, part) loop (in-tree) vs the unrolled chain (build/os0): bits and stage A/B
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in default os0; do
  if [ "$v" = default ]; then lib=$PWD/video-gen-evals_amd/vge/libvge.so; else lib=$PWD/video-gen-evals_amd/csrc/build/$v/libvge.so; fi
  VGE_LIB=$lib timeout -k 10 120 python -u tools/enc_dump.py gpurun_out/dump_$v.npz || exit $?
done
python tools/enc_compare.py gpurun_out/dump_default.npz gpurun_out/dump_os0.npz
bash tools/ab_x3s.sh default os0 2>&1 | grep tag || exit 1
bash tools/ab_x3s.sh default os0 2>&1 | grep tag || exit 1
