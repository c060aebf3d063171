#!/bin/bash
# r06at: the pose extractors' 1x1 convs off the library (one stream-K side only): DWPose / e2e-chain GPU tests, then
# the default bench line with the nested config-3 record
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dwpose.py tests/test_e2e_chain.py -m gpu \
  > gpurun_out/r06at_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06at_tests.log; exit 1; }
tail -1 gpurun_out/r06at_tests.log
timeout -k 10 560 python -u bench.py > gpurun_out/r06at_bench.json 2> gpurun_out/r06at_bench.err || { echo "bench failed"; tail -20 gpurun_out/r06at_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06at_bench.json'));e=d['e2e'];print(d['value'],d['ms_per_step'],d['roofline']['frac'],e.get('value'),e.get('child_wall_s'),e.get('error'))"
