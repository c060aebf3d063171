#!/bin/bash
# Grouped-conv A/B pass: grouped-conv + backbone tests, bitwise detector outputs vs the HEAD kernel (build/gcold),
# interleaved detector timing at the 128-frame chunk over VARIANTS (tools/ab_frcnn.sh names), then the detector trace +
# FETCH_SIZE + WRITE_SIZE passes for the per-layer bytes.  Usage: bash tools/gpu_gconv_ab.sh TAG [VARIANTS...]
set -u
TAG=${1:-r06o}; shift || true; VARIANTS=${*:-default VGE_GC_XCD=0 gcold}
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_frcnn.py -m gpu -k "grouped or backbone" \
  > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 200 python -u tools/frcnn_dump.py gpurun_out/${TAG}_new.pt 64 64 > /dev/null 2>&1 || { echo "dump new failed"; exit 1; }
VGE_LIB=$R/video-gen-evals_amd/csrc/build/gcold/libvge.so timeout -k 10 200 python -u tools/frcnn_dump.py gpurun_out/${TAG}_old.pt 64 64 > /dev/null 2>&1 || { echo "dump old failed"; exit 1; }
python -c "
import torch
a=torch.load('gpurun_out/${TAG}_new.pt');b=torch.load('gpurun_out/${TAG}_old.pt')
print('bitwise', all(torch.equal(a[k],b[k]) for k in ('dets','n_dets','person','n_person')), all(torch.equal(x,y) for x,y in zip(a['fpn'],b['fpn'])))"
rm -f gpurun_out/${TAG}_new.pt gpurun_out/${TAG}_old.pt
CHUNK=128 bash tools/ab_frcnn.sh ${TAG} 2 $VARIANTS || { echo "ab failed"; exit 1; }
for f in gpurun_out/${TAG}_*_[12].json; do python -c "import json;d=json.load(open('$f'));print('$f',round(d['ms_per_pass'],2))"; done
ONLY=frcnn bash tools/profile_e2e.sh ${TAG} || { echo "profile failed"; exit 1; }
python tools/frcnn_layer_bytes.py ${TAG} 128 > gpurun_out/${TAG}_layer_bytes.txt 2>&1 || { echo "layer bytes failed"; exit 1; }
grep -E "conv2|^total|kind:conv2" gpurun_out/${TAG}_layer_bytes.txt | tail -14
