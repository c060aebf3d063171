#!/bin/bash
# The f16 throughput mode at 256 windows: conv_encoder_f16w_kernel vs the staggered single-fp16 x3s kernel.
R="$GRAFT_REPO_ROOT"; cd "$R" && mkdir -p gpurun_out
for r in 1 2; do
  for x in 0 1; do
    VGE_F16_X3S=$x timeout -k 10 240 python -u bench.py --compute f16 --steps 50 --warmup 5 --no-cpu-baseline \
      --no-throughput-mode > gpurun_out/r05x_f16_x${x}_r$r.json 2> gpurun_out/r05x_f16_x${x}_r$r.err || exit 1
  done
done
