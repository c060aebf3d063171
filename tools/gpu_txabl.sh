#!/bin/bash
# transformer ablation builds (tools/build_tx_variant.sh) at 256 windows, f32x3: stage times vs the in-tree library
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/ab_x3s.sh default txabl64 txabl2 txabl1 txabl66 2>&1 | grep tag
