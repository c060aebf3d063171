#!/bin/bash
# Transformer FFN block order rotated per workgroup (default) vs not (frot0): parity, then the bench A/B.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_bench_parity.py tests/test_gpu_parity.py tests/test_nokp_layout.py \
  tests/test_checkpoint_shapes.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05ak_tests.log 2>&1 || exit 1
bash tools/ab_bench_libs.sh 3 default frot0 > gpurun_out/r05ak_ab.log 2>&1 || exit 1
