#!/bin/bash
# r06aa: ROIAlign from an LDS copy of each proposal's feature window (roi_align_win_kernel): detector tests, bitwise
# detector outputs vs the round-start library (build/gcold) with the library GEMM path off on both sides, interleaved
# timing with the window kernel (default) and without it (VGE_ROI_WIN=0), and the per-layer trace
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_frcnn.py \
  > gpurun_out/r06aa_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06aa_tests.log; exit 1; }
tail -1 gpurun_out/r06aa_tests.log
VGE_GEMM_LIB=0 timeout -k 10 200 python -u tools/frcnn_dump.py gpurun_out/r06aa_new.pt 64 64 > /dev/null 2>&1 || { echo "dump new failed"; exit 1; }
VGE_LIB=$R/video-gen-evals_amd/csrc/build/gcold/libvge.so timeout -k 10 200 python -u tools/frcnn_dump.py gpurun_out/r06aa_old.pt 64 64 > /dev/null 2>&1 || { echo "dump old failed"; exit 1; }
python -c "
import torch
a=torch.load('gpurun_out/r06aa_new.pt');b=torch.load('gpurun_out/r06aa_old.pt')
print('bitwise', all(torch.equal(a[k],b[k]) for k in ('dets','n_dets','person','n_person')), all(torch.equal(x,y) for x,y in zip(a['fpn'],b['fpn'])))"
rm -f gpurun_out/r06aa_new.pt gpurun_out/r06aa_old.pt
CHUNK=128 bash tools/ab_frcnn.sh r06aa 2 default VGE_ROI_WIN=0 || { echo "ab failed"; exit 1; }
for f in gpurun_out/r06aa_*_[12].json; do python -c "import json;d=json.load(open('$f'));print('$f',round(d['ms_per_pass'],2))"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r06aa_trace" -o run -- \
  python3 "$R/tools/time_frcnn.py" 128 128 1 > "$R/gpurun_out/r06aa_trace.log" 2>&1 || { echo "trace failed"; exit 1; }
cd "$R" && python tools/frcnn_layers.py "$(find gpurun_out/r06aa_trace -name '*kernel_trace.csv' | sort | tail -1)" > gpurun_out/r06aa_layers.txt 2>&1
grep -E "roi_align|^total" gpurun_out/r06aa_layers.txt | tail -4
