#!/bin/bash
# r06p: featurise with its statistics staged (LDS / one load block) instead of a load behind each store: feats parity
# tests, standalone featurise timing and the config-2 bench line vs the HEAD featurise (build/fzold), interleaved; then
# the grouped-conv / ROIAlign detector pass (tools/gpu_gconv_ab.sh r06o)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_nokp_layout.py tests/test_bench_parity.py > gpurun_out/r06p_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06p_tests.log; exit 1; }
tail -1 gpurun_out/r06p_tests.log
for r in 1 2 3; do
  for v in default fzold; do
    L=$R/video-gen-evals_amd/vge/libvge.so; [ $v = fzold ] && L=$R/video-gen-evals_amd/csrc/build/fzold/libvge.so
    VGE_LIB=$L timeout -k 10 120 python -u tools/time_featurize.py $v 2>/dev/null | tail -1 || exit 1
  done
done
bash tools/ab_bench_libs.sh 3 default fzold || exit 1
bash tools/gpu_gconv_ab.sh r06o default VGE_ROI_OLD=1 VGE_GC_XCD=0 gcold
