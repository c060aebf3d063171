#!/bin/bash
# r06b: persistent GEMM parity + A/B (ViT shapes, detector), chunk guard tests, bench line with the nested config-3 record
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_hmr.py -k "persistent or epilogues" \
  -m gpu > gpurun_out/r06b_tests1.log 2>&1 || { echo "hmr tests failed"; tail -30 gpurun_out/r06b_tests1.log; exit 1; }
tail -2 gpurun_out/r06b_tests1.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_dwpose.py -k "gemm_variant or persistent" \
  -m gpu > gpurun_out/r06b_tests2.log 2>&1 || { echo "dwpose tests failed"; tail -30 gpurun_out/r06b_tests2.log; exit 1; }
tail -2 gpurun_out/r06b_tests2.log
timeout -k 10 240 python -u tools/gemm_bench.py --frames 256 --rounds 5 --waves w8s,p,auto,lib > gpurun_out/r06b_gemm.json 2>&1 || { echo "gemm bench failed"; tail -20 gpurun_out/r06b_gemm.json; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/r06b_gemm.json'))
for k,v in d.items():
  if k!='_check': print(k, {x:round(y,1) for x,y in v.items() if x.endswith('tflops')})
print(d.get('_check'))"
for v in 0 1; do
  VGE_CONV_GEMMP=$v timeout -k 10 180 python -u tools/time_frcnn.py 256 64 2 > gpurun_out/r06b_frcnn_p$v.json 2>/dev/null || { echo "frcnn p$v failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06b_frcnn_p$v.json'));print('gemmp',$v,d['ms_per_pass'],d['backbone_tflops'])"
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_frcnn.py tests/test_hmr.py \
  tests/test_dwpose.py -m gpu > gpurun_out/r06b_tests3.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06b_tests3.log; exit 1; }
tail -2 gpurun_out/r06b_tests3.log
for c in 128 64 128; do
  timeout -k 10 180 python -u tools/time_frcnn.py 256 $c 2 > gpurun_out/r06b_frcnn_c$c.json 2>/dev/null || { echo "frcnn $c failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06b_frcnn_c$c.json'));print('chunk',d['chunk'],d['ms_per_pass'],d['backbone_tflops'])"
done
timeout -k 10 560 python -u bench.py > gpurun_out/r06b_bench.json 2> gpurun_out/r06b_bench.err || { echo "bench failed"; tail -20 gpurun_out/r06b_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06b_bench.json'));e=d.get('e2e',{});print(d['value'],d['ms_per_step'],e.get('value'),e.get('error'),e.get('child_wall_s'))"
