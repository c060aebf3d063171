#!/bin/bash
# Round-5 GPU pass o: featurise without the rotation staging buffer (16 KB of LDS: fits beside a transformer
# workgroup): parity, standalone and in-bench A/B against the previous source (featprev); then pass n.
R="$GRAFT_REPO_ROOT"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_bench_parity.py tests/test_nokp_layout.py -x -q \
  --timeout 200 --timeout-method thread -m gpu > gpurun_out/r05o_tests.log 2>&1 || exit 1
TOOL=featurize bash tools/ab_libs.sh 3 default featprev > gpurun_out/r05o_feat_ab.log 2>&1 || exit 1
bash tools/ab_bench_libs.sh 2 default featprev > gpurun_out/r05o_bench_ab.log 2>&1 || exit 1
bash tools/gpu_r05n.sh || exit 1
bash tools/ab_frcnn.sh r05o 2 default roiprev || exit 1
