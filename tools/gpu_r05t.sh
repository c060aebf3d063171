#!/bin/bash
# Round-5 closing lines: config 3 at 1k clips and config 5, at the HEAD sources (extractor traffic from pmc_e2e r05z).
R="$GRAFT_REPO_ROOT"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --workload e2e --clips 1000 --steps 1 --warmup 1 > gpurun_out/r05t_e2e_cfg3_1k.json \
  2> gpurun_out/r05t_e2e.err || exit 1
timeout -k 10 300 python -u bench.py --workload cfg5 --steps 3 --warmup 1 > gpurun_out/r05t_cfg5.json \
  2> gpurun_out/r05t_cfg5.err || exit 1
