#!/bin/bash
# Round-5 GPU pass g: direct grouped-conv kernel (vge_gconv.hip): detector parity, unit test, timing A/B, layer trace.
R="$GRAFT_REPO_ROOT"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_frcnn.py -x -v -s --timeout 300 --timeout-method thread -m gpu \
  > gpurun_out/r05g_frcnn_tests.log 2>&1 || exit 1
timeout -k 10 240 python -u tools/time_frcnn.py 256 32 2 > gpurun_out/r05g_time_direct.json 2> gpurun_out/r05g_time_direct.err || exit 1
VGE_FRCNN_GCONV=0 timeout -k 10 240 python -u tools/time_frcnn.py 256 32 2 > gpurun_out/r05g_time_gemm.json 2> gpurun_out/r05g_time_gemm.err || exit 1
timeout -k 10 240 python -u tools/time_frcnn.py 256 32 2 > gpurun_out/r05g_time_direct2.json 2> gpurun_out/r05g_time_direct2.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r05g_trace" -o run -- python3 "$R/tools/time_frcnn.py" 64 32 1 \
  > "$R/gpurun_out/r05g_trace.log" 2>&1 || exit 1
