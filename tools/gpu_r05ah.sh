#!/bin/bash
# Detector chunk 96 (below the 32-bit row-offset cap of 104 at 800 px) vs 64, 384 frames, 2 interleaved rounds.
R="$GRAFT_REPO_ROOT"; cd "$R" && mkdir -p gpurun_out
for r in 1 2; do
  for c in 64 96; do
    timeout -k 10 300 python -u tools/time_frcnn.py 384 $c 2 > gpurun_out/r05ah_c${c}_r$r.json 2>/dev/null || exit 1
  done
done
