set -o pipefail
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/rtrace -o rt -- python3 $GRAFT_REPO_ROOT/tools/trace_rtmpose_layers.py > $GRAFT_REPO_ROOT/gpurun_out/rtrace.log 2>&1 && echo TRACE_OK
