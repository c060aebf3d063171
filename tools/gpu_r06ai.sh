#!/bin/bash
# r06ai: 1x1 convs with few input channels on the tuner's kernels instead of hipBLASLt (VGE_LIB_MIN_K = 128 / 256 /
# 512) vs every 1x1 on the library (default): interleaved YOLOX (256-frame chunk) and detector (128-frame chunk) timing;
# first the detector GPU tests (the RPN NMS scan rewritten: bit-scan to the next live box, copy-out after the scan)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_frcnn.py -m gpu \
  > gpurun_out/r06ai_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06ai_tests.log; exit 1; }
tail -1 gpurun_out/r06ai_tests.log
for r in 1 2; do
  for k in 0 128 256 512; do
    VGE_LIB_MIN_K=$k timeout -k 10 200 python -u tools/yolox_prof.py --frames 512 --calls 2 --chunk 256 > gpurun_out/r06ai_yolox_k${k}_$r.json 2>/dev/null || { echo "yolox $k failed"; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r06ai_yolox_k${k}_$r.json'));print('yolox k$k r$r',{a:round(b,2) for a,b in d['stage_ms_per_call'].items()})"
  done
done
CHUNK=128 bash tools/ab_frcnn.sh r06ai 2 default VGE_LIB_MIN_K=128 VGE_LIB_MIN_K=256 VGE_LIB_MIN_K=512 || { echo "ab failed"; exit 1; }
for f in gpurun_out/r06ai_*_[12].json; do case $f in *yolox*) continue;; esac; python -c "import json;d=json.load(open('$f'));print('$f',round(d['ms_per_pass'],2),{k:round(v,2) for k,v in d.get('stage_ms_per_pass',{}).items()})"; done
