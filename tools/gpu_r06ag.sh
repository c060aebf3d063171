#!/bin/bash
# r06ag: separable ROIAlign load-batch shapes: 2 or 4 rows x 4 columns per batch, FMAs of cells outside the support
# skipped (s1) or done on a zero load (s0); box-feature tests per build, interleaved detector timing
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
for v in default br2s0 br4s1 br4s0; do
  L=$R/video-gen-evals_amd/csrc/build/$v/libvge.so; [ $v = default ] && L=$R/video-gen-evals_amd/vge/libvge.so
  VGE_LIB=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_frcnn.py -m gpu -k "box_features or roi_align" \
    > gpurun_out/r06ag_tests_$v.log 2>&1 || { echo "tests $v failed"; tail -30 gpurun_out/r06ag_tests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r06ag_tests_$v.log)"
done
CHUNK=128 bash tools/ab_frcnn.sh r06ag 2 default br2s0 br4s1 br4s0 || { echo "ab failed"; exit 1; }
for f in gpurun_out/r06ag_*_[12].json; do python -c "import json;d=json.load(open('$f'));print('$f',round(d['ms_per_pass'],2),{k:round(v,2) for k,v in d.get('stage_ms_per_pass',{}).items()})"; done
