#!/bin/bash
# transformer parity + per-segment traces (VGE_TRACE build in csrc/build/txtrace) at W = 1 and 2 + stage times
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -m gpu -x -q -s --timeout 120 --timeout-method thread tests/test_bench_parity.py tests/test_gpu_parity.py > gpurun_out/pytest_tx.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_tx.log; [ $rc -le 1 ] || exit $rc
for w in 1 2; do
  VGE_LIB=$PWD/video-gen-evals_amd/csrc/build/txtrace/libvge.so timeout -k 10 120 python -u tools/trace_transformer.py --windows 512 --tx-w $w > gpurun_out/txtrace_w$w.json || exit 1
done
for w in 600 4096; do WINDOWS=$w bash tools/ab_env.sh "w1_$w:VGE_TX_W=1" "w2_$w:VGE_TX_W=2" 2>&1 | grep tag || exit 1; done
