#!/bin/bash
R="$GRAFT_REPO_ROOT"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_frcnn.py -x -v -s --timeout 300 --timeout-method thread -m gpu \
  > gpurun_out/r05j_frcnn_tests.log 2>&1 || exit 1
bash tools/ab_frcnn.sh r05j 2 default gcth8 gcth2 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r05j_trace" -o run -- python3 "$R/tools/time_frcnn.py" 64 32 1 \
  > "$R/gpurun_out/r05j_trace.log" 2>&1 || exit 1
