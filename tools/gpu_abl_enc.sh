#!/bin/bash
# Ablation timings (tools/ablate.sh builds) and the per-phase trace of the conv encoder for one compute mode.
# Usage on the box: bash tools/gpu_abl_enc.sh COMPUTE "ABL masks..."
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
B=video-gen-evals_amd/csrc/build
C=${1:-f32x3}
for A in 0 $2; do
  if [ $A = 0 ]; then L=video-gen-evals_amd/vge/libvge.so; else L=$B/abl$A/libvge.so; fi
  echo "== ABL $A"; VGE_LIB=$L timeout -k 10 120 python -u tools/time_encoder.py --calls 20 --compute $C --tag abl$A 2>&1 | tail -1 || exit 1
done
echo "== trace round 0"; VGE_LIB=$B/trace/libvge.so timeout -k 10 120 python -u tools/trace_encoder.py --compute $C 2>&1 | tail -1
echo "== trace round 2"; VGE_LIB=$B/trace2/libvge.so timeout -k 10 120 python -u tools/trace_encoder.py --compute $C 2>&1 | tail -1
