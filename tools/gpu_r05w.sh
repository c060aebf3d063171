#!/bin/bash
# Config 5: featurise serial vs on the side stream (side3) now that it holds 16 KB of LDS, x the staggered single-fp16
# conv (VGE_F16_X3S=1); 2 interleaved rounds, same box.
R="$GRAFT_REPO_ROOT"; cd "$R" && mkdir -p gpurun_out
for r in 1 2; do
  for p in serial side3; do
    for x in 0 1; do
      VGE_F16_X3S=$x timeout -k 10 240 python -u bench.py --workload cfg5 --steps 3 --warmup 1 --no-cpu-baseline \
        --pipeline $p > gpurun_out/r05w_${p}_x${x}_r$r.json 2> gpurun_out/r05w_${p}_x${x}_$r.err || exit 1
    done
  done
done
