#!/bin/bash
# per-segment trace of transformer_x3_kernel at 256 windows (one window per workgroup), VGE_TRACE build
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
VGE_LIB=$PWD/video-gen-evals_amd/csrc/build/txtrace/libvge.so timeout -k 10 120 python -u tools/trace_transformer.py --windows 256 > gpurun_out/txtrace_256.json && cat gpurun_out/txtrace_256.json
