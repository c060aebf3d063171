#!/bin/bash
# conv kernel MFMA shapes on one box: parity of both (VGE_X3T=1: 16x16x32, 0: 32x32x16) vs the oracle / exact f32,
# then interleaved bench lines of both (driver-style invocation).  Usage: bash tools/gpu_ab_x3t.sh [ROUNDS]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py::test_x3_quad_and_pair_blocks_vs_f32 "tests/test_bench_parity.py::test_bench_workload_vs_oracle" \
  > gpurun_out/pytest_x3t.log 2>&1 && echo X3T_TESTS_OK || { tail -40 gpurun_out/pytest_x3t.log; exit 1; }
for r in $(seq 1 "${1:-2}"); do
  for v in 0 1; do
    VGE_X3T=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-throughput-mode > gpurun_out/bench_x3t${v}_$r.log 2>&1 \
      || { tail -20 gpurun_out/bench_x3t${v}_$r.log; exit 1; }
    python3 - "$v" "$r" <<'PY'
import json, sys
d = json.loads([x for x in open(f"gpurun_out/bench_x3t{sys.argv[1]}_{sys.argv[2]}.log") if x.startswith("{")][-1])
print("x3t", sys.argv[1], "round", sys.argv[2], round(d["value"]), "videos/s, conv", round(d["roofline"]["avg_launch_ms"], 4),
      "ms, frac", round(d["roofline"]["frac"], 3), "dAC", d["precision"]["max_abs_ac"], "dTC", d["precision"]["max_abs_tc"])
PY
  done
done
