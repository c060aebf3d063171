#!/bin/bash
# A/B of environment settings of the in-tree library: encoder stage times (tools/time_encoder.py), interleaved,
# 3 passes.  Usage on the box: bash tools/ab_env.sh "TAG1:VAR=1 VAR2=0" "TAG2:" ...  [WINDOWS env: batch, default 256]
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for pass in 1 2 3; do
  for spec in "$@"; do
    tag=${spec%%:*}; envs=${spec#*:}
    env $envs timeout -k 10 120 python -u tools/time_encoder.py --tag $tag --calls 30 --windows ${WINDOWS:-256} \
      --compute ${COMPUTE:-f32x3} || exit $?
  done
done
