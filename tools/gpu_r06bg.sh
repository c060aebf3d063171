#!/bin/bash
# r06bg: conv2_bf16_kernel on 256 x 128 tiles (variants 13 / 14) as tuner candidates for the 65-128-channel layers:
# bit-identity and DWPose GPU tests, then interleaved YOLOX timing (1,024-frame chunk) with / without them
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dwpose.py -m gpu \
  > gpurun_out/r06bg_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06bg_tests.log; exit 1; }
grep -E "256x128|passed|failed" gpurun_out/r06bg_tests.log | tail -6
for r in 1 2; do
  for v in 1 0; do
    VGE_CONV_C2N=$v timeout -k 10 200 python -u tools/yolox_prof.py --frames 1024 --calls 2 --chunk 1024 > gpurun_out/r06bg_yolox_c2n${v}_$r.json 2>/dev/null || { echo "yolox $v failed"; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r06bg_yolox_c2n${v}_$r.json'));print('c2n=$v r$r',{a:round(b,2) for a,b in d['stage_ms_per_call'].items()})"
  done
  for v in 1 0; do
    VGE_CONV_C2N=$v timeout -k 10 200 python -u tools/time_dwpose.py > gpurun_out/r06bg_dwpose_c2n${v}_$r.json 2>/dev/null || { echo "dwpose $v failed"; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r06bg_dwpose_c2n${v}_$r.json'));print('dwpose c2n=$v r$r',{a:(round(b,2) if isinstance(b,float) else b) for a,b in d.items() if 'ms' in a})"
  done
done
