set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] &&
timeout -k 10 400 python -u bench.py --workload tag --steps 5 --warmup 1 > gpurun_out/bench_tag.log 2>&1 && tail -1 gpurun_out/bench_tag.log | cut -c1-200 && grep -o '"stage_s_last_step_rank0": {[^}]*}' gpurun_out/bench_tag.log
