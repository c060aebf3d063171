#!/bin/bash
# r06g: grouped-conv MFMA loop order (tap-major default vs the old pixel-tile-major build gcord0): bitwise detector
# outputs, grouped-conv tests, interleaved detector timing at the 128-frame chunk
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 200 python -u tools/frcnn_dump.py gpurun_out/r06g_new.pt 64 64 > /dev/null 2>&1 || { echo "dump new failed"; exit 1; }
VGE_LIB=$R/video-gen-evals_amd/csrc/build/gcord0/libvge.so timeout -k 10 200 python -u tools/frcnn_dump.py gpurun_out/r06g_old.pt 64 64 > /dev/null 2>&1 || { echo "dump old failed"; exit 1; }
python -c "
import torch
a=torch.load('gpurun_out/r06g_new.pt');b=torch.load('gpurun_out/r06g_old.pt')
print('bitwise', all(torch.equal(a[k],b[k]) for k in ('dets','n_dets','person','n_person')), all(torch.equal(x,y) for x,y in zip(a['fpn'],b['fpn'])))"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_frcnn.py -m gpu -k "gconv or grouped" > gpurun_out/r06g_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06g_tests.log; exit 1; }
tail -1 gpurun_out/r06g_tests.log
CHUNK=128 bash tools/ab_frcnn.sh r06g 2 default gcord0 || { echo "ab failed"; exit 1; }
for f in gpurun_out/r06g_*_[12].json; do python -c "import json;d=json.load(open('$f'));print('$f',round(d['ms_per_pass'],2))"; done
