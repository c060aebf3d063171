#!/bin/bash
# One GPU pass on the box: pytest -m gpu, smoke(), the default bench line (driver-style invocation), then the
# rocprofv3 kernel trace + PMC passes of the f32x3 headline (tools/profile_round.sh).  Usage:
#   bash tools/gpu_round.sh TAG [pytest selectors...]      (TAG names the profile directories; "-" skips profiling)
set -o pipefail
TAG=${1:--}; shift
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread "${@:-tests}" \
  > gpurun_out/pytest_gpu.log 2>&1 && echo TESTS_OK && tail -1 gpurun_out/pytest_gpu.log || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log || { tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 560 python -u bench.py > gpurun_out/bench.log 2>&1 && echo BENCH_OK && tail -1 gpurun_out/bench.log | cut -c1-600 || { tail -20 gpurun_out/bench.log; exit 1; }
[ "$TAG" = "-" ] && exit 0
bash tools/profile_round.sh "$TAG" f32x3
