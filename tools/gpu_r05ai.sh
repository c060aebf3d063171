#!/bin/bash
# (side4 was an experiment build of bench.py, reverted after this A/B; see profiles/ab_r05ai_pipeline_side4.json)
# Config 2: the transformer's stage time with the featurise overlapped on the side stream (side3, default) vs serial.
R="$GRAFT_REPO_ROOT"; cd "$R" && mkdir -p gpurun_out
for r in 1 2 3 4 5; do
  for p in side4 serial; do
    timeout -k 10 240 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-throughput-mode --pipeline $p \
      > gpurun_out/r05ai_${p}_r$r.json 2> gpurun_out/r05ai_${p}_r$r.err || exit 1
  done
done
