#!/bin/bash
# Kernel trace + stats of a config-3 step (128 clips: every extractor kernel of the e2e chain) for the per-kernel view.
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/pe_r05ag_e2e_trace" -o run \
  -- python3 "$R/bench.py" --workload e2e --clips 128 --steps 1 --warmup 1 --no-cpu-baseline \
  > "$OUT/pe_r05ag_e2e_trace.log" 2>&1
echo "rc=$?"
