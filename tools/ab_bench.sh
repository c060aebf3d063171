#!/bin/bash
# Interleaved A/B of bench.py option sets on one box (the default bench line's workload), ROUNDS passes.
# Usage on the box: bash tools/ab_bench.sh ROUNDS "TAG1:--opt a" "TAG2:--opt b" ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
R=$1; shift
for r in $(seq 1 "$R"); do
  for spec in "$@"; do
    tag=${spec%%:*}; opts=${spec#*:}
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-throughput-mode --no-e2e --steps 50 $opts \
      > gpurun_out/ab_${tag}_$r.log 2>&1 || { tail -20 gpurun_out/ab_${tag}_$r.log; exit 1; }
    python3 - "$tag" "gpurun_out/ab_${tag}_$r.log" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][-1])
st = d.get("stage_ms", {})
print(sys.argv[1], round(d["value"]), "ms/step", round(d["ms_per_step"], 4), "conv", round(d["roofline"]["avg_launch_ms"], 4),
      "tx", round(st.get("transformer", 0), 4), "feat", round(d["featurize"]["avg_ms"], 4), "dAC", d["precision"]["max_abs_ac"])
PY
  done
done
