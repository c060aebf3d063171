#!/bin/bash
# r06w: config 3 end to end (the bench's nested e2e record, standalone) with the library GEMMs
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --workload e2e --clips 1000 --steps 1 --warmup 1 --cpu-seconds 15 > gpurun_out/r06w_e2e.json 2> gpurun_out/r06w_e2e.err || { tail -20 gpurun_out/r06w_e2e.err; exit 1; }
python -c "
import json; d=json.loads([l for l in open('gpurun_out/r06w_e2e.json') if l.startswith('{')][-1])
print(d['value'], d['stage_ms'].get('frcnn_backbone_gemm'), d['gate_detector'])"
