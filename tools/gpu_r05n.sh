#!/bin/bash
# Round-5 GPU pass n: detector tests (chunk cap), then config 3 at 1k clips with the round's detector.
R="$GRAFT_REPO_ROOT"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_frcnn.py tests/test_e2e_chain.py tests/test_hmr_front.py -x -q \
  --timeout 300 --timeout-method thread -m gpu > gpurun_out/r05n_tests.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py --workload e2e --clips 1000 --steps 1 --warmup 1 > gpurun_out/r05n_e2e_cfg3_1k.json \
  2> gpurun_out/r05n_e2e.err || exit 1
