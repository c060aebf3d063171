#!/bin/bash
# rocprofv3 kernel trace + PMC passes of the default bench (f32x3 headline and the f16 throughput mode)
cd "$GRAFT_REPO_ROOT"
bash tools/profile_round.sh r03d f32x3 && bash tools/profile_round.sh r03d16 f16
