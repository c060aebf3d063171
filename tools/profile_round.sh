#!/bin/bash
# Kernel-trace + PMC passes of bench.py on the GPU box (one rocprofv3 run per counter group, no tracing
# domains combined with --pmc).  Usage (from the repo root on the box):
#   bash tools/profile_round.sh TAG [COMPUTE]
# Writes gpurun_out/prof_TAG_{trace,fetch,write,sq,l2}/ ; summarise with tools/pmc_to_json.py.
set -u
TAG=$1
COMPUTE=${2:-f16}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-throughput-mode --no-e2e --compute $COMPUTE"
run() {  # name, extra rocprofv3 args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$OUT/prof_${TAG}_$name" -o run -- python3 $BENCH \
    > "$OUT/prof_${TAG}_$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"
  return $rc
}
run trace --kernel-trace --stats &&
run fetch --pmc FETCH_SIZE --kernel-trace &&
run write --pmc WRITE_SIZE --kernel-trace &&
run l2 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace &&
run sq --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace
