#!/bin/bash
# Per-phase traces of the fp16 unit conv kernel at 256 windows from VGE_TRACE builds (tools/build_variant_src.sh NAME vge_encoder_x3.hip "-DVGE_TRACE"):
# bash tools/trace_f16w.sh trace trace1 ...  (build dirs under video-gen-evals_amd/csrc/build)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in "$@"; do
  VGE_LIB=video-gen-evals_amd/csrc/build/$v/libvge.so timeout -k 10 120 python -u tools/trace_encoder.py \
    --compute f16 --windows 256 > gpurun_out/trace_f16w_$v.json || exit 1
  python3 - "$v" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/trace_f16w_{sys.argv[1]}.json"))
print(sys.argv[1], {w: {k: round(v) for k, v in x.items()} for w, x in d["unit_windows"].items()})
print("  ", {k: v["w0"] for k, v in d.items() if isinstance(v, dict) and "w0" in v and (not k.startswith("conv") or k in ("conv0_stream", "conv0_epi", "conv1_stream", "conv1_epi"))})
PY
done
