set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/p1_trace -o p -- python3 $R/tools/conv1x1_probe.py > $R/gpurun_out/p1_trace.log 2>&1 && echo T_OK &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/p1_fetch -o p -- python3 $R/tools/conv1x1_probe.py > $R/gpurun_out/p1_fetch.log 2>&1 && echo F_OK &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/p1_write -o p -- python3 $R/tools/conv1x1_probe.py > $R/gpurun_out/p1_write.log 2>&1 && echo W_OK &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/p1_sq -o p -- python3 $R/tools/conv1x1_probe.py > $R/gpurun_out/p1_sq.log 2>&1 && echo S_OK
