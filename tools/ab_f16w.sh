#!/bin/bash
# fp16 conv kernels A/B: the 8-wave quad/pair kernel (VGE_F16W=0) vs the 8-wave unit-table kernel with at most 6 or 5
# windows per unit (VGE_F16W=6 / 5), stage times from tools/time_encoder.py at the given window counts.
# Usage on the box: bash tools/ab_f16w.sh "256 4096" [rounds]
cd "$GRAFT_REPO_ROOT"
for r in $(seq 1 ${2:-2}); do
  for n in $1; do
    for cfg in "VGE_F16W=0" "VGE_F16W=6" "VGE_F16W=5"; do
      env $cfg timeout -k 10 120 python -u tools/time_encoder.py --compute f16 --windows $n --tag "$cfg" 2>&1 | tail -1 || exit 1
    done
  done
done
