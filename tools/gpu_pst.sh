#!/bin/bash
# transformer split_rows_e with paired 4-byte stores: parity tests, then same-box bench A/B against the 2-byte stores
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_bench_parity.py tests/test_gpu_parity.py tests/test_nokp_layout.py tests/test_gpu_parity.py > gpurun_out/pst_test.log 2>&1 || { tail -30 gpurun_out/pst_test.log; exit 1; }
tail -2 gpurun_out/pst_test.log
B=video-gen-evals_amd/csrc/build
for r in 1 2 3; do
  for v in pst0 new; do
    lib=$PWD/$B/$v/libvge.so; [ $v = new ] && lib=$PWD/video-gen-evals_amd/vge/libvge.so
    VGE_LIB=$lib timeout -k 10 240 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-throughput-mode > gpurun_out/pst_$v$r.log 2>&1 || { tail -20 gpurun_out/pst_$v$r.log; exit 1; }
    python - "$v$r" gpurun_out/pst_$v$r.log <<'PY'
import json, sys
l = [x for x in open(sys.argv[2]) if x.startswith("{")][-1]
d = json.loads(l)
st = d.get("stage_ms", {})
print(sys.argv[1], round(d["value"]), "ms/step", round(d["ms_per_step"], 4), "conv", round(d["roofline"]["avg_launch_ms"], 4),
      "fuse", st.get("fusion_pool"), "tx", st.get("transformer"), "dAC", d["precision"]["max_abs_ac"])
PY
  done
done
