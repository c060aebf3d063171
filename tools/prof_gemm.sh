#!/bin/bash
# PMC passes over the extractor GEMM (tools/gemm_bench.py --only SHAPE, our kernel only), one rocprofv3 run per
# counter group.  Usage (repo root, GPU box): bash tools/prof_gemm.sh TAG SHAPE [WAVES]   (WAVES: w8 | w4 | w8s | lib)
set -u
TAG=$1; SHAPE=${2:-qkv}; WAVES=${3:-w8}
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 120 rocprofv3 "$@" --output-format csv -d "$OUT/pg_${TAG}_$name" -o run -- python3 "$R/tools/gemm_bench.py" \
    --only "$SHAPE" --waves "$WAVES" --rounds 3 > "$OUT/pg_${TAG}_$name.log" 2>&1
  local rc=$?; echo "[$name] rc=$rc"; return $rc
}
run trace --kernel-trace --stats &&
run sq --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace &&
run fetch --pmc FETCH_SIZE TCC_HIT_sum --kernel-trace &&
run miss --pmc TCC_MISS_sum WRITE_SIZE --kernel-trace &&
run lds --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace
