#!/bin/bash
# tail-stream parity (ragged chunks) + the bench's cross-step score check (score and cfg5 workloads)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_bench_parity.py \
  -k "tail_stream or pipelined" > gpurun_out/steps_test.log 2>&1 || { tail -30 gpurun_out/steps_test.log; exit 1; }
tail -6 gpurun_out/steps_test.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/steps_bench.log 2>&1 || { tail -20 gpurun_out/steps_bench.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/steps_bench.log').read().strip().splitlines()[-1]); print(round(d['value']), d['precision']['last_step_equals_first'], d['throughput_mode']['precision'].get('last_step_equals_first'))"
timeout -k 10 400 python -u bench.py --workload cfg5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/steps_cfg5.log 2>&1 || { tail -20 gpurun_out/steps_cfg5.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/steps_cfg5.log').read().strip().splitlines()[-1]); print(round(d['value']), d['precision']['last_step_equals_first'])"
