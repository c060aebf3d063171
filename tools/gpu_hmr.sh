set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_hmr.py -m gpu -x -v --timeout 200 --timeout-method thread -s > gpurun_out/pytest_hmr.log 2>&1 && echo TESTS_OK &&
timeout -k 10 300 python -u tools/time_hmr.py --frames 64 --iters 3 > gpurun_out/time_hmr.log 2>&1 && echo TIME_OK && cat gpurun_out/time_hmr.log
