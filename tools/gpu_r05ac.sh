#!/bin/bash
# gconv3: the next two images' tiles in flight (PF 2) vs one: unit tests, then the detector A/B at chunk 64
# (default = PF 2 for group widths >= 32; VGE_GC_PF=1 / 2 force one depth everywhere).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_frcnn.py -m gpu -x -q -k grouped --timeout 120 --timeout-method thread \
  > gpurun_out/r05ac_tests.log 2>&1 || exit 1
VGE_GC_PF=2 timeout -k 10 300 python -u -m pytest tests/test_frcnn.py -m gpu -x -q -k grouped --timeout 120 \
  --timeout-method thread > gpurun_out/r05ac_tests_pf2.log 2>&1 || exit 1
CHUNK=64 bash tools/ab_frcnn.sh r05ac 2 default VGE_GC_PF=1 VGE_GC_PF=2 || exit 1
