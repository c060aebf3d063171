set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_yolox.py tests/test_dwpose.py -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_yolox.log 2>&1 && echo YOLOX_TESTS_OK
