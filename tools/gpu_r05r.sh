#!/bin/bash
# 16x16x32 for every bf16-output GEMM epilogue (the 1x1 convs' too): ViT shapes + detector A/B + extractor tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_bench.py --waves w8,w8s,auto,lib --rounds 7 > gpurun_out/r05r_gemm.json 2> gpurun_out/r05r_gemm.err || exit 1
timeout -k 10 600 python -u -m pytest tests/test_hmr.py tests/test_dwpose.py tests/test_frcnn.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r05r_tests.log 2>&1 || exit 1
CHUNK=64 bash tools/ab_frcnn.sh r05r 2 default gw8 || exit 1
