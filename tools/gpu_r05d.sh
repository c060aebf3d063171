#!/bin/bash
# Round-5 GPU pass d: staggered single-fp16 conv (VGE_F16_X3S=1) parity + config-5 A/B; transformer chunk rotation A/B.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
VGE_F16_X3S=1 timeout -k 10 300 python -u -m pytest tests/test_bench_parity.py tests/test_gpu_parity.py -x -q \
  --timeout 120 --timeout-method thread -m gpu -k "f16 and not unit_table" > gpurun_out/r05d_f16x3s_parity.log 2>&1 || exit 1
for k in 1 2; do
  timeout -k 10 240 python bench.py --workload cfg5 --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/r05d_cfg5_base$k.json 2> gpurun_out/r05d_cfg5_base$k.err || exit 1
  VGE_F16_X3S=1 timeout -k 10 240 python bench.py --workload cfg5 --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/r05d_cfg5_x3s$k.json 2> gpurun_out/r05d_cfg5_x3s$k.err || exit 1
done
COMPUTE=f32x3 WINDOWS=256 bash tools/ab_libs.sh 2 default txrot1 txrot4 > gpurun_out/r05d_txrot.log 2>&1 || exit 1
