#!/bin/bash
# r06al: the fused stem with weights as the row operand (8-B stem-value stores), separate patch / stem LDS regions, two
# barriers per tile, vs the two kernels (VGE_STEM_FUSED=0): tests, then interleaved detector timing
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 120 python -u -m pytest -x -s -q --timeout 100 --timeout-method thread tests/test_frcnn.py -m gpu -k stem_pool \
  > gpurun_out/r06al_stem_test.log 2>&1 || { echo "stem test failed"; tail -40 gpurun_out/r06al_stem_test.log; exit 1; }
grep -E "P[2-6]:|passed|failed" gpurun_out/r06al_stem_test.log
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_frcnn.py tests/test_e2e_chain.py -m gpu \
  > gpurun_out/r06al_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06al_tests.log; exit 1; }
tail -1 gpurun_out/r06al_tests.log
CHUNK=128 bash tools/ab_frcnn.sh r06al 2 default VGE_STEM_FUSED=0 || { echo "ab failed"; exit 1; }
for f in gpurun_out/r06al_*_[12].json; do python -c "import json;d=json.load(open('$f'));print('$f',round(d['ms_per_pass'],2),{k:round(v,2) for k,v in d.get('stage_ms_per_pass',{}).items()})"; done
