#!/bin/bash
# SQ counters of the gate detector's kernels (one 64-frame chunk after a warm call): MFMA busy / wait split per kernel.
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pe_r05u_frcnn_sq" -o run \
  -- python3 "$R/tools/time_frcnn.py" 64 64 1 > "$OUT/pe_r05u_frcnn_sq.log" 2>&1
echo "rc=$?"
