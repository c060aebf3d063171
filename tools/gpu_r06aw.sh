#!/bin/bash
# r06aw: config 4 end to end at the round's final extractor sources (2-rank GPU test vs the oracle flow; the 1-GPU bench line)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_tag_e2e.py -m gpu \
  > gpurun_out/r06aw_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06aw_tests.log; exit 1; }
grep -E "config-4|passed|failed" gpurun_out/r06aw_tests.log | tail -3
timeout -k 10 500 python -u bench.py --workload tag --extract --steps 1 --warmup 1 > gpurun_out/r06aw_tag_e2e.json \
  2> gpurun_out/r06aw_tag_e2e.err || { echo "tag e2e failed"; tail -20 gpurun_out/r06aw_tag_e2e.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06aw_tag_e2e.json'));print(d['value'],d['ms_per_step'],d['rank0_last_step'],d['videos_scored'],d['cpu_baseline']['value'])"
