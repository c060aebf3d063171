#!/bin/bash
# end-of-session check on one box: pytest -m gpu, smoke(), the default bench line (driver-style invocation)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log || { tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 > gpurun_out/bench50.log 2>&1 && tail -1 gpurun_out/bench50.log | cut -c1-300
