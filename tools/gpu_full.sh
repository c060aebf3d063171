set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo TESTS_OK && tail -1 gpurun_out/pytest_gpu.log &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 && echo BENCH_OK && tail -1 gpurun_out/bench.log | cut -c1-300 &&
timeout -k 10 400 python -u bench.py --workload tag --steps 3 --warmup 1 > gpurun_out/bench_tag.log 2>&1 && tail -1 gpurun_out/bench_tag.log | cut -c1-200 && grep -o '"stage_s_last_step_rank0": {[^}]*}' gpurun_out/bench_tag.log
