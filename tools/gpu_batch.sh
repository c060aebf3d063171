#!/bin/bash
# Run several GPU step scripts in one box session: bash tools/gpu_batch.sh "script1 args" "script2 args" ...
# A step's ordinary failure (exit 1/2) moves on to the next; a time limit, abort, fault or kill (124, 134, 137, 139,
# or any status >= 128) ends the batch there.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for step in "$@"; do
  echo "=== $step"
  bash $step
  rc=$?
  echo "=== rc=$rc"
  if [ $rc -ge 124 ] && [ $rc -ne 126 ] && [ $rc -ne 127 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
