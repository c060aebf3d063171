#!/bin/bash
# r06bb: the gate detector's workspace with aliased buffers (stem output, upsample, RPN conv output, ROI features):
# detector / e2e-chain GPU tests, then config 3 with 2,048-frame extraction passes (out of memory before)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_frcnn.py tests/test_e2e_chain.py -m gpu \
  > gpurun_out/r06bb_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06bb_tests.log; exit 1; }
tail -1 gpurun_out/r06bb_tests.log
for cc in 64 32; do
  timeout -k 10 450 python -u bench.py --workload e2e --clips 1000 --steps 1 --warmup 1 --cpu-seconds 2 --chunk-clips $cc > gpurun_out/r06bb_cc$cc.json 2> gpurun_out/r06bb_cc$cc.err || { echo "e2e $cc failed"; grep -v amdgpu.ids gpurun_out/r06bb_cc$cc.err | tail -5; continue; }
  python -c "import json;e=json.load(open('gpurun_out/r06bb_cc$cc.json'));print('chunk-clips $cc',e['value'],e['ms_per_step'],round(e['frames_per_s'],1),{k:round(v,1) for k,v in e['stage_ms'].items()})"
done
