#!/bin/bash
# Parity + bench + profile passes on the box: the conv / bench parity tests, the default bench line, then
# tools/profile_round.sh for the given modes.  Usage: bash tools/gpu_check_prof.sh TAG [MODES...] (default f32x3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=$1; shift
MODES=${@:-f32x3}
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_bench_parity.py > gpurun_out/pytest_$TAG.log 2>&1 || { tail -20 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1 || { tail -5 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-200
for m in $MODES; do
  bash tools/profile_round.sh ${TAG}$m $m || exit 1
done
