#!/bin/bash
# Refresh the extractor PMC at HEAD (the grouped conv changed), then the config-3 line at 1k clips.
R="$GRAFT_REPO_ROOT"; cd "$R" && mkdir -p gpurun_out
bash tools/profile_e2e.sh r05al || exit 1
timeout -k 10 900 python -u bench.py --workload e2e --clips 1000 --steps 1 --warmup 1 > gpurun_out/r05al_e2e_cfg3_1k.json \
  2> gpurun_out/r05al_e2e.err || exit 1
