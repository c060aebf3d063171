#!/bin/bash
# r06ah: YOLOX-L per-layer times at HEAD (256-frame chunk, the e2e bench's chunk): rocprofv3 kernel trace of one
# detect call, paired with the layer list (tools/yolox_layers.py)
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06ah_yolox -o run -- python tools/yolox_prof.py --frames 256 --calls 1 --chunk 256 \
  > gpurun_out/r06ah_prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r06ah_prof.log; exit 1; }
python tools/yolox_layers.py gpurun_out/r06ah_yolox 256 > gpurun_out/r06ah_yolox_layers.txt 2>&1 || { cat gpurun_out/r06ah_yolox_layers.txt | tail; exit 1; }
cat gpurun_out/r06ah_yolox_layers.txt
