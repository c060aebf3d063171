#!/bin/bash
# r06e: config-3 extractor PMC / kernel-trace passes at the round-6 sources (tools/profile_e2e.sh r06e)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash tools/profile_e2e.sh r06e
