#!/bin/bash
# r06r: config-3 extractor PMC / kernel-trace passes at the round-6 grouped-conv sources (tools/profile_e2e.sh r06r)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash tools/profile_e2e.sh r06r
