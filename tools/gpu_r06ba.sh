#!/bin/bash
# r06ba: config 3 extraction-pass size: 1,024 frames (default) vs 2,048 (--chunk-clips 64), same box
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
for cc in 32 64; do
  timeout -k 10 450 python -u bench.py --workload e2e --clips 1000 --steps 1 --warmup 1 --cpu-seconds 2 --chunk-clips $cc > gpurun_out/r06ba_cc$cc.json 2> gpurun_out/r06ba_cc$cc.err || { echo "e2e $cc failed"; grep -v amdgpu.ids gpurun_out/r06ba_cc$cc.err | tail -20; exit 1; }
  python -c "import json;e=json.load(open('gpurun_out/r06ba_cc$cc.json'));print('chunk-clips $cc',e['value'],e['ms_per_step'],round(e['frames_per_s'],1),{k:round(v,1) for k,v in e['stage_ms'].items()})"
done
