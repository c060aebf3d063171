#!/bin/bash
# Round-5 GPU pass h: grouped conv with GC_NI images per workgroup: parity, A/B against 1 / 2, layer trace.
R="$GRAFT_REPO_ROOT"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_frcnn.py -x -v -s --timeout 300 --timeout-method thread -m gpu \
  > gpurun_out/r05h_frcnn_tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in default gcni1 gcni2; do
    if [ $v = default ]; then L=$R/video-gen-evals_amd/vge/libvge.so; else L=$R/video-gen-evals_amd/csrc/build/$v/libvge.so; fi
    VGE_LIB=$L timeout -k 10 240 python -u tools/time_frcnn.py 256 32 2 > gpurun_out/r05h_time_${v}_$r.json 2>/dev/null || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r05h_trace" -o run -- python3 "$R/tools/time_frcnn.py" 64 32 1 \
  > "$R/gpurun_out/r05h_trace.log" 2>&1 || exit 1
