set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_bench.py --rounds 5 > gpurun_out/gemm_bench.log 2>&1 && cat gpurun_out/gemm_bench.log
