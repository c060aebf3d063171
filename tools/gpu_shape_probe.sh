#!/bin/bash
# MFMA shape probe (tools/probes/mfma_shape_probe.hip, built in-tree): 32x32x16 vs 16x16x32 f16 in the split stream's loop
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 ./tools/probes/mfma_shape_probe 200000 8 > gpurun_out/shape_probe.json 2>&1; rc=$?; cat gpurun_out/shape_probe.json; exit $rc
