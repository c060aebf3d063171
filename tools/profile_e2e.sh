#!/bin/bash
# Config-3 extractor profiles on the GPU box (one rocprofv3 run per pass; no tracing domains with --pmc):
#   hmr_{fetch,write}    PMC of the TokenHMR extractor alone (tools/time_hmr.py, full ViT-H/16, 256 frames x 3 calls)
#   yolox_{trace,fetch,write}  kernel trace + stats and PMC of the detector on one e2e pass (tools/yolox_prof.py,
#                        1,024 frames in one 1,024-frame chunk, the e2e bench's, 2 profiled calls)
#   frcnn_{trace,fetch,write}  kernel trace + stats and PMC of the gate detector (tools/time_frcnn.py, 256 frames in
#                        one 256-frame chunk, the product's: a warm call + 1 timed call; the counters of the timed call)
# Summarise with tools/pmc_e2e.py TAG (-> profiles/pmc_e2e.json) and tools/yolox_prof_check.py.
#   Usage (repo root, GPU box): bash tools/profile_e2e.sh TAG   (ONLY=frcnn: the three frcnn passes only)
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {  # name, script args (as one string), extra rocprofv3 args...
  local name=$1 cmd=$2; shift 2
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$OUT/pe_${TAG}_$name" -o run -- python3 $cmd \
    > "$OUT/pe_${TAG}_$name.log" 2>&1
  local rc=$?; echo "[$name] rc=$rc"; return $rc
}
HMR="$R/tools/time_hmr.py --frames 256 --iters 2"
YOLOX="$R/tools/yolox_prof.py --frames 1024 --calls 2 --chunk 1024"
FRCNN="$R/tools/time_frcnn.py 256 256 1"
run frcnn_trace "$FRCNN" --kernel-trace --stats &&
run frcnn_fetch "$FRCNN" --pmc FETCH_SIZE --kernel-trace &&
run frcnn_write "$FRCNN" --pmc WRITE_SIZE --kernel-trace &&
{ [ "${ONLY:-}" = frcnn ] && exit 0; true; } &&
run yolox_trace "$YOLOX" --kernel-trace --stats &&
run yolox_fetch "$YOLOX" --pmc FETCH_SIZE --kernel-trace &&
run yolox_write "$YOLOX" --pmc WRITE_SIZE --kernel-trace &&
run hmr_fetch "$HMR" --pmc FETCH_SIZE --kernel-trace &&
run hmr_write "$HMR" --pmc WRITE_SIZE --kernel-trace
