#!/bin/bash
# config-5 bench line (10k 64-frame clips, f16, 4,096-window chunks) on the box
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --workload cfg5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/cfg5.log 2>&1 && echo CFG5_OK &&
python3 -c "import json; d=json.loads(open('gpurun_out/cfg5.log').read().strip().splitlines()[-1]); print(d['value'], d.get('stage_ms'), d.get('precision', {}).get('max_abs_ac'), d['roofline']['frac'])"
