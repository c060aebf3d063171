#!/bin/bash
# ROIAlign with XCD-contiguous frames (default) vs the plain order (roiplain): detector tests + A/B at chunk 64.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_frcnn.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r05ab_tests.log 2>&1 || exit 1
CHUNK=64 bash tools/ab_frcnn.sh r05ab 2 default roiplain || exit 1
