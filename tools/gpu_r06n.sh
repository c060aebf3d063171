#!/bin/bash
# r06n: grouped conv in XCD-contiguous workgroup order (gc_xcd) on top of r06m's per-shape tiles: grouped-conv tests,
# bitwise detector outputs vs the HEAD kernel (build/gcold), interleaved detector timing at the 128-frame chunk
# (new / new in launch order / old), then the detector's trace + FETCH_SIZE + WRITE_SIZE passes for the per-layer bytes
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_frcnn.py -m gpu -k "grouped or backbone" \
  > gpurun_out/r06n_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06n_tests.log; exit 1; }
tail -1 gpurun_out/r06n_tests.log
timeout -k 10 200 python -u tools/frcnn_dump.py gpurun_out/r06n_new.pt 64 64 > /dev/null 2>&1 || { echo "dump new failed"; exit 1; }
VGE_LIB=$R/video-gen-evals_amd/csrc/build/gcold/libvge.so timeout -k 10 200 python -u tools/frcnn_dump.py gpurun_out/r06n_old.pt 64 64 > /dev/null 2>&1 || { echo "dump old failed"; exit 1; }
python -c "
import torch
a=torch.load('gpurun_out/r06n_new.pt');b=torch.load('gpurun_out/r06n_old.pt')
print('bitwise', all(torch.equal(a[k],b[k]) for k in ('dets','n_dets','person','n_person')), all(torch.equal(x,y) for x,y in zip(a['fpn'],b['fpn'])))"
rm -f gpurun_out/r06n_new.pt gpurun_out/r06n_old.pt
CHUNK=128 bash tools/ab_frcnn.sh r06n 2 default VGE_GC_XCD=0 gcold || { echo "ab failed"; exit 1; }
for f in gpurun_out/r06n_*_[12].json; do python -c "import json;d=json.load(open('$f'));print('$f',round(d['ms_per_pass'],2))"; done
ONLY=frcnn bash tools/profile_e2e.sh r06n || { echo "profile failed"; exit 1; }
python tools/frcnn_layer_bytes.py r06n 128 > gpurun_out/r06n_layer_bytes.txt 2>&1 || { echo "layer bytes failed"; exit 1; }
grep -E "conv2|^total|kind:conv2" gpurun_out/r06n_layer_bytes.txt | tail -14
