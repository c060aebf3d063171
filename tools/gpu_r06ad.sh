#!/bin/bash
# r06ad: grouped conv with two images' tile loads in flight (VGE_GC_PD=2) and / or 8 images per workgroup
# (VGE_GC_NI=8): grouped-conv tests on the default build, interleaved detector timing over the builds
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_frcnn.py -m gpu -k "grouped or backbone" \
  > gpurun_out/r06ad_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06ad_tests.log; exit 1; }
tail -1 gpurun_out/r06ad_tests.log
for v in pd2 ni8 pd2ni8; do
  VGE_LIB=$R/video-gen-evals_amd/csrc/build/$v/libvge.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_frcnn.py -m gpu -k "grouped" > gpurun_out/r06ad_tests_$v.log 2>&1 || { echo "tests $v failed"; tail -20 gpurun_out/r06ad_tests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r06ad_tests_$v.log)"
done
CHUNK=128 bash tools/ab_frcnn.sh r06ad 2 default pd2 ni8 pd2ni8 || { echo "ab failed"; exit 1; }
for f in gpurun_out/r06ad_*_[12].json; do python -c "import json;d=json.load(open('$f'));print('$f',round(d['ms_per_pass'],2))"; done
