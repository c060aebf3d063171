set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/time_flow_setup.py > gpurun_out/flow_setup.log 2>&1; rc=$?; cat gpurun_out/flow_setup.log; exit $rc
