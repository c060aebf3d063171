#!/bin/bash
# config-3 line at its 1k clips (gate on), then the detector alone under rocprofv3 --kernel-trace (cross-check of the
# yolox stage's GEMM rate)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --workload e2e --clips 1000 --steps 1 --warmup 1 > gpurun_out/e2e_1k.log 2>&1 && echo E2E1K_OK || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/yolox_prof_trace -o run -- python3 $GRAFT_REPO_ROOT/tools/yolox_prof.py > $GRAFT_REPO_ROOT/gpurun_out/yolox_prof.log 2>&1 && echo YPROF_OK
