#!/bin/bash
# gemm2 (two 128 x 256 workgroups per CU, register epilogue) vs the 256 x 256 kernel: bitwise check + timing at the
# ViT-H shapes, then the extractor tests with VGE_GEMM_WAVES=2 (every GEMM and 1x1-conv-as-GEMM through gemm2).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_bench.py --waves w8,w8s,w2,lib --rounds 7 > gpurun_out/r05q_gemm.json 2> gpurun_out/r05q_gemm.err || exit 1
VGE_GEMM_WAVES=2 timeout -k 10 600 python -u -m pytest tests/test_hmr.py tests/test_dwpose.py tests/test_frcnn.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r05q_tests_w2.log 2>&1 || exit 1
