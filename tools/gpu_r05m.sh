#!/bin/bash
# Round-5 GPU pass m: detector chunk size (frames per workspace pass: activations in the 256 MB MALL or not).
R="$GRAFT_REPO_ROOT"; cd "$R" && mkdir -p gpurun_out
for c in 128 256; do
  timeout -k 10 300 python -u tools/time_frcnn.py 256 $c 2 > gpurun_out/r05m_chunk$c.json 2> gpurun_out/r05m_chunk$c.err || exit 1
done
