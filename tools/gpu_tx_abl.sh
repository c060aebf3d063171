#!/bin/bash
# per-segment transformer traces of ablation builds (csrc/build/tx*/): W = 1 and 2 at 512 windows
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in "$@"; do for w in 1 2; do
  VGE_LIB=$PWD/video-gen-evals_amd/csrc/build/$v/libvge.so timeout -k 10 120 python -u tools/trace_transformer.py --windows 512 --tx-w $w > gpurun_out/txabl_${v}_w$w.json || exit 1
done; done
