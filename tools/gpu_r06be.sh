#!/bin/bash
# r06be: the separable ROIAlign's sample-loop branch forced for every ROI vs roi_align_kernel (bit-identical), and the
# detector / e2e-chain GPU tests
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_frcnn.py tests/test_e2e_chain.py -m gpu \
  > gpurun_out/r06be_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06be_tests.log; exit 1; }
grep -E "roi_align|passed|failed" gpurun_out/r06be_tests.log | tail -3
