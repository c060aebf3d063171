#!/bin/bash
# conv kernel ring depths (X3S_PF_QUAD / X3S_PF_PAIR): same-box bench A/B of variant builds
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
B=video-gen-evals_amd/csrc/build
for r in 1 2; do
  for v in new pp12 pp6 pq3; do
    lib=$PWD/$B/$v/libvge.so; [ $v = new ] && lib=$PWD/video-gen-evals_amd/vge/libvge.so
    VGE_LIB=$lib timeout -k 10 240 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-throughput-mode > gpurun_out/pf_$v$r.log 2>&1 || { tail -20 gpurun_out/pf_$v$r.log; exit 1; }
    python - "$v$r" gpurun_out/pf_$v$r.log <<'PY'
import json, sys
l = [x for x in open(sys.argv[2]) if x.startswith("{")][-1]
d = json.loads(l)
st = d.get("stage_ms", {})
print(sys.argv[1], round(d["value"]), "ms/step", round(d["ms_per_step"], 4), "conv", round(d["roofline"]["avg_launch_ms"], 4),
      "fuse", st.get("fusion_pool"), "tx", st.get("transformer"), "dAC", d["precision"]["max_abs_ac"])
PY
  done
done
