#!/bin/bash
# r06m: grouped conv with per-shape output tiles (gc_pick_tile) and 3 workgroups per CU at group widths <= 32:
# grouped-conv + detector tests, bitwise detector outputs vs the HEAD kernel (build/gcold), interleaved detector timing
# at the 128-frame chunk (new / new with the legacy 4 x 32 tile / old), and one kernel trace for the per-layer times
set -u
R="${GRAFT_REPO_ROOT:-$(pwd)}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_frcnn.py -m gpu \
  > gpurun_out/r06m_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r06m_tests.log; exit 1; }
tail -1 gpurun_out/r06m_tests.log
timeout -k 10 200 python -u tools/frcnn_dump.py gpurun_out/r06m_new.pt 64 64 > /dev/null 2>&1 || { echo "dump new failed"; exit 1; }
VGE_LIB=$R/video-gen-evals_amd/csrc/build/gcold/libvge.so timeout -k 10 200 python -u tools/frcnn_dump.py gpurun_out/r06m_old.pt 64 64 > /dev/null 2>&1 || { echo "dump old failed"; exit 1; }
python -c "
import torch
a=torch.load('gpurun_out/r06m_new.pt');b=torch.load('gpurun_out/r06m_old.pt')
print('bitwise', all(torch.equal(a[k],b[k]) for k in ('dets','n_dets','person','n_person')), all(torch.equal(x,y) for x,y in zip(a['fpn'],b['fpn'])))"
rm -f gpurun_out/r06m_new.pt gpurun_out/r06m_old.pt
CHUNK=128 bash tools/ab_frcnn.sh r06m 2 default VGE_GC_TILE=legacy gcold || { echo "ab failed"; exit 1; }
for f in gpurun_out/r06m_*_[12].json; do python -c "import json;d=json.load(open('$f'));print('$f',round(d['ms_per_pass'],2))"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r06m_trace" -o run -- \
  python3 "$R/tools/time_frcnn.py" 128 128 1 > "$R/gpurun_out/r06m_trace.log" 2>&1 || { echo "trace failed"; exit 1; }
cd "$R" && python tools/frcnn_layers.py "$(find gpurun_out/r06m_trace -name '*kernel_trace.csv' | sort | tail -1)" > gpurun_out/r06m_layers.txt 2>&1
grep -E "conv2|total" gpurun_out/r06m_layers.txt | tail -12
