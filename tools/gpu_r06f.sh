#!/bin/bash
# r06f: SQ / memory counters of the persistent GEMM vs the one-tile kernel on the ViT qkv shape
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; OUT=$R/gpurun_out; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CMD="$R/tools/gemm_bench.py --only qkv --waves w8s,p --rounds 2"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/gp_r06f_sq" -o run -- python3 $CMD > "$OUT/gp_r06f_sq.log" 2>&1 && echo sq ok &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/gp_r06f_fetch" -o run -- python3 $CMD > "$OUT/gp_r06f_fetch.log" 2>&1 && echo fetch ok &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d "$OUT/gp_r06f_write" -o run -- python3 $CMD > "$OUT/gp_r06f_write.log" 2>&1 && echo write ok
