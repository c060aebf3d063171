#!/bin/bash
# Interleaved A/B of libvge.so builds through the default bench line (bench.py --steps 50, no CPU baseline / f16 mode),
# ROUNDS passes.  A build is "default" (the in-tree library) or a variant under video-gen-evals_amd/csrc/build/
# (tools/build_variant_src.sh NAME SOURCE.hip "-DFOO=1").  Usage on the box: bash tools/ab_bench_libs.sh ROUNDS default varA ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
R=$1; shift
for r in $(seq 1 "$R"); do
  for v in "$@"; do
    case $v in
      default) L=$PWD/video-gen-evals_amd/vge/libvge.so ;;
      *) L=$PWD/video-gen-evals_amd/csrc/build/$v/libvge.so ;;
    esac
    VGE_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-throughput-mode --no-e2e --steps 50 \
      > gpurun_out/abl_${v}_$r.log 2>&1 || { tail -20 gpurun_out/abl_${v}_$r.log; exit 1; }
    python3 - "$v" "gpurun_out/abl_${v}_$r.log" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][-1])
print(sys.argv[1], round(d["value"]), "ms/step", round(d["ms_per_step"], 4), "conv", round(d["roofline"]["avg_launch_ms"], 4),
      "tx", round(d["stage_ms"]["transformer"], 4), "dAC", d["precision"]["max_abs_ac"])
PY
  done
done
