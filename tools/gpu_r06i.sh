#!/bin/bash
# r06i: scores written by the score kernel straight into pinned host memory (--host-scores direct) vs two copy kernels
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bench_parity.py -m gpu \
  -k "pinned or deferred or tail or side_stream" > gpurun_out/r06i_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06i_tests.log; exit 1; }
tail -1 gpurun_out/r06i_tests.log
for r in 1 2 3; do
  for h in copy direct; do
    timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-throughput-mode --no-e2e \
      --host-scores $h > gpurun_out/r06i_${h}_$r.json 2>/dev/null || { echo "bench $h failed"; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r06i_${h}_$r.json'));print('$h',$r,round(d['value']),round(d['ms_per_step'],4),d['precision']['last_step_equals_first'],d['precision']['max_abs_ac'])"
  done
done
