#!/bin/bash
# r06ax: extractor chunk sizes at the final sources: YOLOX 256 / 512 / 1,024 frames per pass (tools/yolox_prof.py,
# 1,024 frames per call) and the gate detector 128 / 256 frames per chunk (tools/time_frcnn.py, 256 frames), interleaved
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
for r in 1 2; do
  for c in 256 512 1024; do
    timeout -k 10 200 python -u tools/yolox_prof.py --frames 1024 --calls 2 --chunk $c > gpurun_out/r06ax_yolox_c${c}_$r.json 2>/dev/null || { echo "yolox $c failed"; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r06ax_yolox_c${c}_$r.json'));print('yolox chunk $c r$r',{a:round(b,2) for a,b in d['stage_ms_per_call'].items()})"
  done
  for c in 128 256; do
    timeout -k 10 240 python -u tools/time_frcnn.py 256 $c 2 > gpurun_out/r06ax_frcnn_c${c}_$r.json 2>/dev/null || { echo "frcnn $c failed"; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r06ax_frcnn_c${c}_$r.json'));print('frcnn chunk $c r$r',round(d['ms_per_pass'],2))"
  done
done
