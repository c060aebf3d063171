#!/bin/bash
# single-fp16 transformer: one window per workgroup at 1 or 2 workgroups per CU vs two windows per workgroup
cd "$GRAFT_REPO_ROOT"
for w in 256 1024 4096; do
  COMPUTE=f16 WINDOWS=$w bash tools/ab_env.sh "w1occ1_$w:VGE_F16_MIX=0 VGE_TX_W=1 VGE_TX_OCC=1" \
    "w1occ2_$w:VGE_F16_MIX=0 VGE_TX_W=1 VGE_TX_OCC=2" "w2_$w:VGE_F16_MIX=0 VGE_TX_W=2" 2>&1 | grep tag || exit 1
done
