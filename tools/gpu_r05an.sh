#!/bin/bash
# (auto_kr0 / vge_debug_set_gemm_krot existed only in the experiment build; see profiles/ab_r05an_gemm_krot.json)
# ViT GEMM with the per-workgroup K rotation (auto) vs without (auto_kr0), then the TokenHMR / e2e tests with it.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_bench.py --waves auto,auto_kr0,lib --rounds 7 > gpurun_out/r05an_gemm.json \
  2> gpurun_out/r05an_gemm.err || exit 1
timeout -k 10 500 python -u -m pytest tests/test_hmr.py tests/test_e2e_chain.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/r05an_tests.log 2>&1 || exit 1
