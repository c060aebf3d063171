set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_dwpose.py -m gpu -k "persistent or conv_bf16" > gpurun_out/pytest_tall.log 2>&1 && tail -5 gpurun_out/pytest_tall.log &&
timeout -k 10 300 python -u tools/conv_bench.py > gpurun_out/conv_bench.log 2>&1 && cat gpurun_out/conv_bench.log &&
timeout -k 10 300 python -u tools/time_dwpose.py --frames 256 --iters 3 --detector > gpurun_out/time_dwpose.log 2>&1 && cat gpurun_out/time_dwpose.log
