#!/bin/bash
# r06c: every GPU test + smoke at HEAD, then the config-5 line (CPU baseline + PMC traffic at the current f16 conv hash)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r06c_gpu_tests.log 2>&1 \
  || { echo "tests failed"; tail -40 gpurun_out/r06c_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r06c_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06c_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r06c_smoke.log; exit 1; }
tail -1 gpurun_out/r06c_smoke.log
timeout -k 10 400 python -u bench.py --workload cfg5 --steps 3 --warmup 1 > gpurun_out/r06c_cfg5.json 2> gpurun_out/r06c_cfg5.err \
  || { echo "cfg5 failed"; tail -20 gpurun_out/r06c_cfg5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06c_cfg5.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['traffic'],d['cpu_baseline']['value'],d['stage_ms'])"
