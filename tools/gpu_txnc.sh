#!/bin/bash
# CLS dot partial sums (build/txnc2, txnc4) vs one chain (in-tree), 256 windows f32x3 and 4,096 single fp16, then the
# transformer parity tests against the 4-sum variant
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/ab_x3s.sh default txnc2 txnc4 2>&1 | grep tag || exit 1
for pass in 1 2; do for v in default txnc4; do
  if [ "$v" = default ]; then lib=$PWD/video-gen-evals_amd/vge/libvge.so; else lib=$PWD/video-gen-evals_amd/csrc/build/$v/libvge.so; fi
  VGE_LIB=$lib VGE_F16_MIX=0 timeout -k 10 120 python -u tools/time_encoder.py --tag ${v}_f16_4096 --calls 10 --windows 4096 --compute f16 || exit $?
done; done
VGE_LIB=$PWD/video-gen-evals_amd/csrc/build/txnc4/libvge.so timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 240 --timeout-method thread tests/test_bench_parity.py > gpurun_out/pytest_txnc.log 2>&1; tail -2 gpurun_out/pytest_txnc.log
