#!/bin/bash
# GEMM first-wave stagger experiment (half the CUs start their tile sequence late by N x 8k cycles).
# (ran on the experiment build of commit history before "Record: GEMM first-wave stagger"; the stagger was not kept)
R="$GRAFT_REPO_ROOT"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u tools/gemm_bench.py --waves auto,auto+1,auto+3,auto+6,lib --rounds 7 \
  > gpurun_out/r05aa_gemm.json 2> gpurun_out/r05aa_gemm.err || exit 1
