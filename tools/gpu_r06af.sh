#!/bin/bash
# r06af: ROIAlign separable form with 8 cell loads in flight per batch (buffer loads, OOB = 0) vs the sample order
# (VGE_ROI_SEP=0): the detector and e2e-chain GPU tests, then interleaved detector timing (128-frame chunks)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_frcnn.py tests/test_e2e_chain.py -m gpu \
  > gpurun_out/r06af_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06af_tests.log; exit 1; }
grep -E "PASS|FAIL|bins identical" gpurun_out/r06af_tests.log | tail -30
CHUNK=128 bash tools/ab_frcnn.sh r06af 2 default VGE_ROI_SEP=0 || { echo "ab failed"; exit 1; }
for f in gpurun_out/r06af_*_[12].json; do python -c "import json;d=json.load(open('$f'));print('$f',round(d['ms_per_pass'],2),{k:round(v,2) for k,v in d.get('stage_ms_per_pass',{}).items()})"; done
