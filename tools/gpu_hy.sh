#!/bin/bash
# skip code only in blocks 2-3 (in-tree) vs skip code everywhere (build/rg) vs the pre-row-group kernel (x3s_old)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in default rg; do
  if [ "$v" = default ]; then lib=$PWD/video-gen-evals_amd/vge/libvge.so; else lib=$PWD/video-gen-evals_amd/csrc/build/$v/libvge.so; fi
  VGE_LIB=$lib timeout -k 10 120 python -u tools/enc_dump.py gpurun_out/dump_$v.npz || exit $?
done
python tools/enc_compare.py gpurun_out/dump_default.npz gpurun_out/dump_rg.npz
bash tools/ab_x3s.sh default rg x3s_old 2>&1 | grep tag || exit 1
bash tools/ab_x3s.sh default rg x3s_old 2>&1 | grep tag || exit 1
