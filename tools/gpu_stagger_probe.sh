#!/bin/bash
# staggered-halves probe (tools/probes/stagger_probe.hip, built in-tree): both MFMA shapes with epilogue-like partners
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 200 ./tools/probes/stagger_probe 1500 3 > gpurun_out/stagger_probe.json 2>&1; rc=$?; cat gpurun_out/stagger_probe.json; exit $rc
