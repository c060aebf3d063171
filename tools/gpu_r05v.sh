#!/bin/bash
# gconv3 on 16x16x32 (VGE_GC_MF=1, default) vs 16x16x16: unit tests vs torch, detector tests, A/B at chunk 64.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_frcnn.py tests/test_e2e_chain.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r05v_tests.log 2>&1 || exit 1
VGE_GC_MF=0 timeout -k 10 200 python -u -m pytest tests/test_frcnn.py -m gpu -x -q -k grouped --timeout 120 \
  --timeout-method thread > gpurun_out/r05v_tests_mf0.log 2>&1 || exit 1
CHUNK=64 bash tools/ab_frcnn.sh r05v 2 default VGE_GC_MF=0 || exit 1
