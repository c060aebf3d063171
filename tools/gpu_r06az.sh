#!/bin/bash
# r06az: the default bench line at HEAD (nested config 3 with YOLOX over the whole pass and 256-frame detector chunks)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 560 python -u bench.py > gpurun_out/r06az_bench.json 2> gpurun_out/r06az_bench.err || { echo "bench failed"; grep -v amdgpu.ids gpurun_out/r06az_bench.err | tail -20; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06az_bench.json'));e=d['e2e'];print(d['value'],d['ms_per_step'],d['roofline']['frac'],e.get('value'),e.get('child_wall_s'),e.get('error'),e['gate_detector']['traffic_per_call'],e['roofline']['traffic'],e.get('yolox_traffic_per_call'))"
