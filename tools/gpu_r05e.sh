#!/bin/bash
# Round-5 GPU pass e: chunk rotation in the conv (X3S_ROT) and transformer (VGE_TX_ROT): parity, A/B, bench, cfg5.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_bench_parity.py -x -q --timeout 120 \
  --timeout-method thread -m gpu > gpurun_out/r05e_parity.log 2>&1 || exit 1
COMPUTE=f32x3 WINDOWS=256 bash tools/ab_libs.sh 3 default x3srot0 txrot0 > gpurun_out/r05e_ab.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r05e_bench.json 2> gpurun_out/r05e_bench.err || exit 1
VGE_F16_X3S=1 timeout -k 10 240 python bench.py --workload cfg5 --steps 3 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r05e_cfg5_x3s.json 2> gpurun_out/r05e_cfg5_x3s.err || exit 1
timeout -k 10 240 python bench.py --workload cfg5 --steps 3 --warmup 1 --no-cpu-baseline \
  > gpurun_out/r05e_cfg5_base.json 2> gpurun_out/r05e_cfg5_base.err || exit 1
