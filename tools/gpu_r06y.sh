#!/bin/bash
# r06y: conv2_bf16_kernel on v_mfma_f32_16x16x32_bf16 (variant 12, a tuner candidate): bit-identity tests, then
# interleaved timing with it (default) and without it (VGE_CONV_SH=0): the gate detector, YOLOX-L alone, DWPose
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_dwpose.py \
  > gpurun_out/r06y_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06y_tests.log; exit 1; }
tail -1 gpurun_out/r06y_tests.log
CHUNK=128 bash tools/ab_frcnn.sh r06y 2 default VGE_CONV_SH=0 || { echo "ab failed"; exit 1; }
for f in gpurun_out/r06y_*_[12].json; do python -c "import json;d=json.load(open('$f'));print('$f',round(d['ms_per_pass'],2), round(d['backbone_tflops']))"; done
for r in 1 2; do for v in 1 0; do
  VGE_CONV_SH=$v timeout -k 10 300 python -u tools/yolox_prof.py --frames 1024 --calls 2 --chunk 256 > gpurun_out/r06y_yolox_${v}_$r.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads([l for l in open('gpurun_out/r06y_yolox_${v}_$r.json') if l.startswith('{')][-1]);print('yolox SH=$v', {k:(round(x,2) if isinstance(x,float) else x) for k,x in d.items() if not isinstance(x,(dict,list))}, d.get('stage_ms'))"
done; done
