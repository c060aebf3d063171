#!/bin/bash
# Detector gate calibration, then a short e2e bench with the calibrated shift.  Usage: bash tools/gpu_e2e_gate.sh [CLIPS]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/yolox_gate_calib.py 1024 > gpurun_out/calib.log 2>&1 && tail -1 gpurun_out/calib.log &&
SHIFT=$(python -c "import json; print(json.load(open('gpurun_out/yolox_gate_calib.json'))['obj_shift'])") &&
VGE_GATE_OBJ_SHIFT=$SHIFT timeout -k 10 600 python -u bench.py --workload e2e --clips ${1:-64} --steps 2 --warmup 1 \
  --no-cpu-baseline > gpurun_out/e2e_gate.log 2>&1 && echo E2E_OK && tail -1 gpurun_out/e2e_gate.log
