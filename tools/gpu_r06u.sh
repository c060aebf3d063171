#!/bin/bash
# r06u: the extractors' bias / residual linears and 1x1 convs on hipBLASLt (vge_blaslt.cpp): library-path tests, the
# detector / TokenHMR / DWPose / e2e-chain GPU tests, then interleaved timing of the gate detector and TokenHMR with the
# library path on (default) and off (VGE_GEMM_LIB=0)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_hmr.py tests/test_frcnn.py \
  tests/test_dwpose.py tests/test_e2e_chain.py > gpurun_out/r06u_tests.log 2>&1 || { echo "tests failed"; grep -E "PASS|FAIL|Error|error" gpurun_out/r06u_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r06u_tests.log; grep -E "max \|lib" gpurun_out/r06u_tests.log | head -20
CHUNK=128 bash tools/ab_frcnn.sh r06u 2 default VGE_GEMM_LIB=0 || { echo "ab failed"; exit 1; }
for f in gpurun_out/r06u_*_[12].json; do python -c "import json;d=json.load(open('$f'));print('$f',round(d['ms_per_pass'],2), round(d['backbone_tflops']), round(d['head_tflops']))"; done
for r in 1 2; do for v in default 0; do
  VGE_GEMM_LIB=$([ $v = 0 ] && echo 0 || echo 1) timeout -k 10 300 python -u tools/time_hmr.py --frames 256 --iters 2 > gpurun_out/r06u_hmr_${v}_$r.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads([l for l in open('gpurun_out/r06u_hmr_${v}_$r.json') if l.startswith('{')][-1]);print('hmr $v $r', {k:(round(x,3) if isinstance(x,float) else x) for k,x in d.items() if not isinstance(x,(dict,list))})"
done; done
