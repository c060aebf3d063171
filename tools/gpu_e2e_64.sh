#!/bin/bash
# config-3 line at 64 clips (gate on): the e2e bench path check
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --workload e2e --clips 64 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/e2e_64.log 2>&1 && echo E2E64_OK &&
python3 -c "import json; d=json.loads(open('gpurun_out/e2e_64.log').read().strip().splitlines()[-1]); print(d['value'], d['front_end']['single_person_fraction'], d['front_end']['videos_accepted_fraction'], d['front_end']['tokenhmr_frames_per_video'], d['yolox_gemm_tflops'], d['roofline']['frac'])"
