#!/bin/bash
# Interleaved A/B timing of two libvge.so builds (stage times from tools/time_encoder.py), per compute mode.
# Usage on the box: bash tools/ab_encoder.sh LIB_A LIB_B "f16 f32x3" [rounds]
cd "$GRAFT_REPO_ROOT"
for r in $(seq 1 ${4:-2}); do
  for c in $3; do
    for L in "$1" "$2"; do
      VGE_LIB=$L timeout -k 10 120 python -u tools/time_encoder.py --compute $c --tag "$c $(basename $(dirname $L))" 2>&1 | tail -1 || exit 1
    done
  done
done
