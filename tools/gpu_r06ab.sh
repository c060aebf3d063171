#!/bin/bash
# r06ab: YOLOX / RTMPose 1x1 SiLU convs (and any-width 1x1s) on the library path: DWPose / e2e-chain tests, then
# interleaved YOLOX-L and DWPose timing with the library path on (default) and off (VGE_GEMM_LIB=0)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_dwpose.py tests/test_e2e_chain.py \
  > gpurun_out/r06ab_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06ab_tests.log; exit 1; }
tail -1 gpurun_out/r06ab_tests.log
for r in 1 2; do for v in 1 0; do
  VGE_GEMM_LIB=$v timeout -k 10 300 python -u tools/yolox_prof.py --frames 1024 --calls 2 --chunk 256 > gpurun_out/r06ab_yolox_${v}_$r.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads([l for l in open('gpurun_out/r06ab_yolox_${v}_$r.json') if l.startswith('{')][-1]);print('yolox lib=$v', d.get('gemm_tflops'), d.get('stage_ms'))"
  VGE_GEMM_LIB=$v timeout -k 10 300 python -u tools/time_dwpose.py > gpurun_out/r06ab_dwpose_${v}_$r.json 2>/dev/null || exit 1
  python -c "import json;ls=[json.loads(l) for l in open('gpurun_out/r06ab_dwpose_${v}_$r.json') if l.startswith('{')];print('dwpose lib=$v', [{k:(round(x,3) if isinstance(x,float) else x) for k,x in d.items() if not isinstance(x,(dict,list))} for d in ls])"
done; done
