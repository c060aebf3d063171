#!/bin/bash
# row-group tiling + tap skipping (in-tree) vs no skipping (build/noskip) vs the previous kernel (build/x3s_old):
# stage A/B, output comparison, round-1 / round-2 traces, conv parity tests
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in default noskip x3s_old; do
  if [ "$v" = default ]; then lib=$PWD/video-gen-evals_amd/vge/libvge.so; else lib=$PWD/video-gen-evals_amd/csrc/build/$v/libvge.so; fi
  VGE_LIB=$lib timeout -k 10 120 python -u tools/enc_dump.py gpurun_out/dump_$v.npz || exit $?
done
python tools/enc_compare.py gpurun_out/dump_default.npz gpurun_out/dump_x3s_old.npz
python tools/enc_compare.py gpurun_out/dump_noskip.npz gpurun_out/dump_x3s_old.npz
bash tools/ab_x3s.sh default noskip x3s_old 2>&1 | grep tag || exit 1
for v in trace_s1 trace_s2; do
  VGE_LIB=$PWD/video-gen-evals_amd/csrc/build/$v/libvge.so timeout -k 10 200 python -u tools/trace_x3s.py > gpurun_out/rg_$v.log 2>&1 || exit $?
  echo "== $v"; sed -n 3,45p gpurun_out/rg_$v.log
done
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_bench_parity.py tests/test_nokp_layout.py > gpurun_out/pytest_rg.log 2>&1; tail -2 gpurun_out/pytest_rg.log
