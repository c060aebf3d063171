#!/bin/bash
# r06ac: config-3 extractor PMC / kernel-trace passes at the round-6 final extractor sources (tools/profile_e2e.sh r06ac)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash tools/profile_e2e.sh r06ac
