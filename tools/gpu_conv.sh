set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dwpose.py tests/test_yolox.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1 && echo TESTS_OK &&
timeout -k 10 300 python -u tools/conv_bench.py > gpurun_out/conv_bench.log 2>&1 && cat gpurun_out/conv_bench.log &&
timeout -k 10 300 python -u tools/time_dwpose.py --frames 256 --iters 3 --detector > gpurun_out/time_dwpose.log 2>&1 && cat gpurun_out/time_dwpose.log
