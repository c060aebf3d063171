set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/conv_bench.py > gpurun_out/conv_bench.log 2>&1 && cat gpurun_out/conv_bench.log
