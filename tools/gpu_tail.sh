#!/bin/bash
# tail-stream pipeline: parity test, then bench A/B (side vs tail), alternating, same box
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -n "$RUN_TEST" ]; then
  timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_bench_parity.py -k "tail_stream or pipelined" > gpurun_out/tail_test.log 2>&1 || { tail -30 gpurun_out/tail_test.log; exit 1; }
  tail -4 gpurun_out/tail_test.log
fi
for r in 1 2; do
  for p in side side2 tailx; do
    timeout -k 10 240 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-throughput-mode --pipeline $p > gpurun_out/tail_$p$r.log 2>&1 || { tail -20 gpurun_out/tail_$p$r.log; exit 1; }
    python - "$p$r" gpurun_out/tail_$p$r.log <<'PY'
import json, sys
l = [x for x in open(sys.argv[2]) if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[1], round(d["value"]), "ms/step", round(d["ms_per_step"], 4), "conv", round(d["roofline"]["avg_launch_ms"], 4))
PY
  done
done
