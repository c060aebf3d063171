cd $GRAFT_REPO_ROOT
for w in 1024 4096; do COMPUTE=f16 WINDOWS=$w bash tools/ab_env.sh "f16m0w1_$w:VGE_F16_MIX=0 VGE_TX_W=1" "f16m0w2_$w:VGE_F16_MIX=0 VGE_TX_W=2" 2>&1 | grep tag || exit 1; done
WINDOWS=2048 bash tools/ab_env.sh "x3w1_2048:VGE_TX_W=1" "x3w2_2048:VGE_TX_W=2" 2>&1 | grep tag
