#!/bin/bash
# x3s A/B on the box: conv parity tests, phase traces of rounds 0 / 2 (trace_s, trace_s2), stage times of the
# in-tree library vs csrc/build/base (interleaved)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_bench_parity.py -k "bench_workload or config5" > gpurun_out/pytest_x3s.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_x3s.log; [ $rc -le 1 ] || exit $rc
for v in trace_s trace_s2; do
  VGE_LIB=$PWD/video-gen-evals_amd/csrc/build/$v/libvge.so timeout -k 10 200 python -u tools/trace_x3s.py > gpurun_out/$v.log 2>&1 || exit $?
  sed -n 3p gpurun_out/$v.log
done
bash tools/ab_x3s.sh default base 2>&1 | grep tag
