#!/bin/bash
# r06aj: RPN NMS mask over the upper triangle with the division skipped for disjoint pairs; the 1x1 library path from
# Cin >= 128 (VGE_LIB_MIN_K default): detector / e2e-chain / DWPose GPU tests, then interleaved detector timing against
# the previous NMS build (build/nms0)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_frcnn.py tests/test_e2e_chain.py tests/test_dwpose.py -m gpu \
  > gpurun_out/r06aj_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06aj_tests.log; exit 1; }
tail -1 gpurun_out/r06aj_tests.log
CHUNK=128 bash tools/ab_frcnn.sh r06aj 2 default nms0 || { echo "ab failed"; exit 1; }
for f in gpurun_out/r06aj_*_[12].json; do python -c "import json;d=json.load(open('$f'));print('$f',round(d['ms_per_pass'],2),{k:round(v,2) for k,v in d.get('stage_ms_per_pass',{}).items()})"; done
