set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_hmr.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_hmr.log 2>&1 && echo TESTS_OK && tail -2 gpurun_out/pytest_hmr.log &&
timeout -k 10 200 python -u tools/gemm_bench.py --waves w8,lib > gpurun_out/gemm_bench.log 2>&1 && cat gpurun_out/gemm_bench.log &&
timeout -k 10 300 python -u tools/time_hmr.py --frames 256 --iters 3 > gpurun_out/time_hmr.log 2>&1 && echo TIME_OK && cat gpurun_out/time_hmr.log
