#!/bin/bash
# the CLS row on an MFMA tile at one window per workgroup (build/txclsm) vs the VALU dot products (in-tree), 256 and
# 600 windows f32x3, then the transformer parity tests against the variant
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/ab_x3s.sh default txclsm 2>&1 | grep tag || exit 1
for pass in 1 2; do for v in default txclsm; do
  if [ "$v" = default ]; then lib=$PWD/video-gen-evals_amd/vge/libvge.so; else lib=$PWD/video-gen-evals_amd/csrc/build/$v/libvge.so; fi
  VGE_LIB=$lib timeout -k 10 120 python -u tools/time_encoder.py --tag ${v}_600 --calls 20 --windows 600 || exit $?
done; done
VGE_LIB=$PWD/video-gen-evals_amd/csrc/build/txclsm/libvge.so timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 240 --timeout-method thread tests/test_bench_parity.py > gpurun_out/pytest_txclsm.log 2>&1; tail -2 gpurun_out/pytest_txclsm.log
