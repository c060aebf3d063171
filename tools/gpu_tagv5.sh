set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_dist_cpu.py tests/test_report.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_tag.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_tag.log; [ $rc -eq 0 ] &&
timeout -k 10 400 python -u bench.py --workload tag --steps 10 --warmup 2 > gpurun_out/bench_tag.log 2>&1 && tail -1 gpurun_out/bench_tag.log | cut -c1-200 && grep -o '"stage_s_last_step_rank0": {[^}]*}' gpurun_out/bench_tag.log
