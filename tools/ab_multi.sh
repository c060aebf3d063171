#!/bin/bash
# Interleaved timing of several libvge.so builds (tools/time_encoder.py stage times) for one compute mode.
# Usage on the box: bash tools/ab_multi.sh COMPUTE ROUNDS LIB...
cd "$GRAFT_REPO_ROOT"
C=$1; R=$2; shift 2
for r in $(seq 1 $R); do
  for L in "$@"; do
    VGE_LIB=$L timeout -k 10 120 python -u tools/time_encoder.py --compute $C --tag "$(basename $(dirname $L))" 2>&1 | tail -1 || exit 1
  done
done
