#!/bin/bash
# The staggered single-fp16 conv as the f16 default: every encoder / flow GPU test, then the config-5 line.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_bench_parity.py tests/test_gpu_parity.py tests/test_stats_cache.py \
  tests/test_checkpoint_shapes.py tests/test_nokp_layout.py tests/test_dist_gpu.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/r05y_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload cfg5 --steps 3 --warmup 1 > gpurun_out/r05y_cfg5.json \
  2> gpurun_out/r05y_cfg5.err || exit 1
