#!/bin/bash
# GEMM ablation pass: where the ViT-H GEMM's time goes (VGE_GABL builds from tools/ablate_gemm.sh), hipBLASLt beside
# each run as the same-process reference.
set -o pipefail
mkdir -p gpurun_out
for A in 0 1 2 4 8; do
  VGE_LIB=tools/abl/libvge_gabl$A.so timeout -k 10 240 python -u tools/gemm_bench.py --waves w8,w8s,lib --rounds 5 \
    > gpurun_out/r05p_gabl$A.json 2> gpurun_out/r05p_gabl$A.err || exit 1
done
