#!/bin/bash
# r06ay: config 3 with the larger extractor chunks (YOLOX 1,024 frames, the gate detector 256): the e2e workload alone
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 450 python -u bench.py --workload e2e --clips 1000 --steps 1 --warmup 1 --cpu-seconds 15 > gpurun_out/r06ay_e2e.json 2> gpurun_out/r06ay_e2e.err || { echo "e2e failed"; grep -v amdgpu.ids gpurun_out/r06ay_e2e.err | tail -20; exit 1; }
python -c "import json;e=json.load(open('gpurun_out/r06ay_e2e.json'));print(e['value'],e['ms_per_step'],{k:round(v,1) for k,v in e['stage_ms'].items()}, e['frames_per_s'])"
