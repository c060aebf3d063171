#!/bin/bash
# Interleaved A/B of libvge.so builds on the gate detector (tools/time_frcnn.py, 256 frames, chunk 32, 2 passes):
# "default" = the in-tree library, "gwN" = the in-tree library with VGE_GEMM_WAVES=N, "VAR=VAL" = the in-tree
# library with that environment variable set, else a variant name under
# video-gen-evals_amd/csrc/build/; CHUNK (env, default 32) = frames per detector chunk.  Usage on the box:
#   bash tools/ab_frcnn.sh TAG ROUNDS default varA ...   -> gpurun_out/TAG_<variant>_<round>.json
R="$GRAFT_REPO_ROOT"; cd "$R" && mkdir -p gpurun_out
TAG=$1; N=$2; shift 2
for r in $(seq 1 "$N"); do
  for v in "$@"; do
    GW=""; XV=VGE_UNUSED_AB; XVAL=""
    if [ "$v" = default ]; then L=$R/video-gen-evals_amd/vge/libvge.so
    elif [ "${v:0:2}" = gw ]; then L=$R/video-gen-evals_amd/vge/libvge.so; GW=${v:2}
    elif [[ "$v" == *=* ]]; then L=$R/video-gen-evals_amd/vge/libvge.so; XV=${v%%=*}; XVAL=${v#*=}
    else L=$R/video-gen-evals_amd/csrc/build/$v/libvge.so; fi
    export "$XV=$XVAL"
    VGE_GEMM_WAVES=$GW VGE_LIB=$L timeout -k 10 240 python -u tools/time_frcnn.py 256 ${CHUNK:-32} 2 \
      > gpurun_out/${TAG}_${v}_$r.json 2>/dev/null || exit 1
    unset "$XV"
  done
done
