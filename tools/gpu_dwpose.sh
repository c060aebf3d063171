set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dwpose.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_dwpose.log 2>&1 && echo DWPOSE_TESTS_OK
