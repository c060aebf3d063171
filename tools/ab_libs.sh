#!/bin/bash
# Interleaved A/B of libvge.so builds: encoder stage times (tools/time_encoder.py; TOOL=featurize: the standalone
# featurise time, tools/time_featurize.py), ROUNDS passes over the builds.
# A build is a path, "default" (the in-tree library) or a variant name under video-gen-evals_amd/csrc/build/
# (tools/build_variant_src.sh NAME SOURCE.hip "-DFOO=1").  Usage on the box:
#   COMPUTE=f32x3 WINDOWS=256 bash tools/ab_libs.sh ROUNDS default varA varB ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
R=$1; shift
for r in $(seq 1 "$R"); do
  for v in "$@"; do
    case $v in
      default) L=$PWD/video-gen-evals_amd/vge/libvge.so ;;
      /*) L=$v ;;
      *) L=$PWD/video-gen-evals_amd/csrc/build/$v/libvge.so ;;
    esac
    if [ "${TOOL:-encoder}" = featurize ]; then
      VGE_LIB=$L timeout -k 10 120 python -u tools/time_featurize.py "$v" || exit 1
    else
      VGE_LIB=$L timeout -k 10 120 python -u tools/time_encoder.py --compute "${COMPUTE:-f32x3}" \
        --windows "${WINDOWS:-256}" --calls 30 --tag "$v" || exit 1
    fi
  done
done
