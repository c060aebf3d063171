#!/bin/bash
# A/B of the extractor GEMM on the two MFMA shapes (32x32x16 vs 16x16x32), ViT-H shapes, plus the output check
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_bench.py --frames 256 --rounds 7 --waves w8,w8s,lib > gpurun_out/gemm16.json 2> gpurun_out/gemm16.err
rc=$?; tail -5 gpurun_out/gemm16.err; cat gpurun_out/gemm16.json; exit $rc
