#!/bin/bash
# Round-5 GPU pass f: transformer ring depth at the rotated chunk order; f16 conv PMC passes at HEAD.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
COMPUTE=f32x3 WINDOWS=256 bash tools/ab_libs.sh 3 default txpf8 > gpurun_out/r05f_txpf.log 2>&1 || exit 1
bash tools/profile_round.sh r05f f16 > gpurun_out/r05f_prof.log 2>&1 || exit 1
