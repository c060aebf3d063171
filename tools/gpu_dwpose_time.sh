set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/time_dwpose.py --frames 256 --iters 3 --detector > gpurun_out/time_dwpose.log 2>&1 && cat gpurun_out/time_dwpose.log &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_dwpose -o dw -- python3 $GRAFT_REPO_ROOT/tools/time_dwpose.py --frames 256 --iters 2 --detector > $GRAFT_REPO_ROOT/gpurun_out/prof_dwpose.log 2>&1 && echo PROF_OK
