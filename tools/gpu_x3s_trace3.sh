#!/bin/bash
# x3s phase traces of rounds 0, 1 (light quads, cold / warm) and 2 (vit pairs) at 256 windows (VGE_TRACE variants)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in trace_s trace_s1 trace_s2; do
  VGE_LIB=$PWD/video-gen-evals_amd/csrc/build/$v/libvge.so timeout -k 10 200 python -u tools/trace_x3s.py > gpurun_out/$v.log 2>&1 || exit $?
  sed -n 3p gpurun_out/$v.log
done
