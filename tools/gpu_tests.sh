#!/bin/bash
# GPU test pass on the box: pytest -m gpu (optionally only files / -k expression given as arguments), then the
# bench line.  Usage: bash tools/gpu_tests.sh [pytest selectors...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 240 --timeout-method thread "${@:-tests}" \
  > gpurun_out/pytest_gpu.log 2>&1 && echo TESTS_OK && tail -1 gpurun_out/pytest_gpu.log &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 && echo BENCH_OK && tail -1 gpurun_out/bench.log | cut -c1-400
