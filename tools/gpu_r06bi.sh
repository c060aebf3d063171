#!/bin/bash
# r06bi: config-3 extractor PMC / kernel-trace passes at the final extractor sources (tools/profile_e2e.sh r06bi)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash tools/profile_e2e.sh r06bi
