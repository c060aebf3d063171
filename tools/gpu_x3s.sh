#!/bin/bash
# x3s bring-up on the box: parity tests, then the bench line (no CPU baseline)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_bench_parity.py \
  > gpurun_out/pytest_x3s.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_x3s.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-throughput-mode > gpurun_out/bench_x3s.log 2>&1 && tail -1 gpurun_out/bench_x3s.log | cut -c1-300
