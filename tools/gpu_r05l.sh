#!/bin/bash
# Round-5 GPU pass k: 1x1 convs on the GEMM kernel (tuner candidate, variant 9): bitwise / parity tests, detector A/B
# (VGE_CONV_GEMM=0 off), ViT GEMM unchanged (vitprev = the previous vge_vit.hip), layer trace.
R="$GRAFT_REPO_ROOT"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dwpose.py tests/test_hmr.py tests/test_frcnn.py -x -q --timeout 300 \
  --timeout-method thread -m gpu > gpurun_out/r05l_tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 240 python -u tools/time_frcnn.py 256 32 2 > gpurun_out/r05l_gemm_$r.json 2>/dev/null || exit 1
  VGE_CONV_GEMM=0 timeout -k 10 240 python -u tools/time_frcnn.py 256 32 2 > gpurun_out/r05l_conv_$r.json 2>/dev/null || exit 1
done
for v in default vitprev; do
  if [ $v = default ]; then L=$R/video-gen-evals_amd/vge/libvge.so; else L=$R/video-gen-evals_amd/csrc/build/$v/libvge.so; fi
  VGE_LIB=$L timeout -k 10 240 python -u tools/time_hmr.py --frames 256 --iters 5 > gpurun_out/r05l_hmr_$v.json 2>/dev/null || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r05l_trace" -o run -- python3 "$R/tools/time_frcnn.py" 64 32 1 \
  > "$R/gpurun_out/r05l_trace.log" 2>&1 || exit 1
