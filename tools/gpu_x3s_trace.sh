#!/bin/bash
# x3s iteration on the box: phase trace (VGE_TRACE variant), bench line (no CPU baseline), optional parity tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
VGE_LIB=$PWD/video-gen-evals_amd/csrc/build/trace_s/libvge.so timeout -k 10 200 python -u tools/trace_x3s.py > gpurun_out/trace_x3s.log 2>&1 || exit $?
tail -29 gpurun_out/trace_x3s.log | cut -c1-110
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-throughput-mode > gpurun_out/bench_x3s.log 2>&1 || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/bench_x3s.log').read().strip().splitlines()[-1]); print(d['value'], d['stage_ms'], d['precision']['max_abs_ac'], d['precision']['max_abs_tc'])"
if [ "$1" = "tests" ]; then
  timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_bench_parity.py > gpurun_out/pytest_x3s.log 2>&1; tail -2 gpurun_out/pytest_x3s.log
fi
