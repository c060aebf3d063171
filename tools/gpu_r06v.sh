#!/bin/bash
# r06v: config-3 extractor PMC / kernel-trace passes at the round-6 library-GEMM sources (tools/profile_e2e.sh r06v)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash tools/profile_e2e.sh r06v
