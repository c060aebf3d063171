#!/bin/bash
# r06a: detector chunk guard (64-bit GEMM epilogue), the default bench line with the nested config-3 record, chunk A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_frcnn.py tests/test_hmr.py \
  tests/test_dwpose.py -m gpu > gpurun_out/r06a_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06a_tests.log; exit 1; }
tail -3 gpurun_out/r06a_tests.log
timeout -k 10 560 python -u bench.py > gpurun_out/r06a_bench.json 2> gpurun_out/r06a_bench.err || { echo "bench failed"; tail -20 gpurun_out/r06a_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06a_bench.json'));e=d.get('e2e',{});print(d['value'],d['ms_per_step'],e.get('value'),e.get('error'),e.get('child_wall_s'))"
for c in 64 128 64 128; do
  timeout -k 10 180 python -u tools/time_frcnn.py 256 $c 2 > gpurun_out/r06a_frcnn_c$c.json 2>/dev/null || { echo "frcnn $c failed"; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06a_frcnn_c$c.json'));print('chunk',d['chunk'],d['ms_per_pass'],d['backbone_tflops'])"
done
