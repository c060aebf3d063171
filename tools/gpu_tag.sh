#!/bin/bash
# config-4 flow bench line (300 videos, full eval flow, CPU baseline = the oracle flow on the same files)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --workload tag --steps 5 --warmup 2 > gpurun_out/tag.log 2>&1 && echo TAG_OK &&
python3 -c "import json; d=json.loads(open('gpurun_out/tag.log').read().strip().splitlines()[-1]); print(d['value'], d['cpu_baseline'])"
