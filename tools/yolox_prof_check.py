#!/usr/bin/env python3
"""Compare tools/yolox_prof.py's hipEvents GEMM stage with a rocprofv3 kernel trace of the same run.

    python tools/yolox_prof_check.py gpurun_out/yolox_prof_trace gpurun_out/yolox_prof.log

The profiled calls are the last `calls` x `chunks_per_call` letterbox_focus dispatches onward (one per 64-frame chunk);
their conv kernels (everything but letterbox / SPP pooling / upsample / decode + NMS) are summed per call.
"""
import csv
import glob
import json
import sys

trace_dir, log = sys.argv[1], sys.argv[2]
info = json.loads([l for l in open(log).read().splitlines() if l.startswith("{")][-1])
rows = []
for f in glob.glob(f"{trace_dir}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
lb = [i for i, r in enumerate(rows) if "letterbox_focus" in r["Kernel_Name"]]
first = lb[-info["calls"] * info["chunks_per_call"]]
other = ("letterbox_focus", "spp_", "upsample2x", "yolox_decode_nms")
conv_ns = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[first:]
              if not any(o in r["Kernel_Name"] for o in other))
other_ns = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[first:]
               if any(o in r["Kernel_Name"] for o in other))
per_call = conv_ns / info["calls"] / 1e6
res = {"rocprof_conv_ms_per_call": per_call, "hipevents_gemm_ms_per_call": info["stage_ms_per_call"]["gemm"],
       "rocprof_other_ms_per_call": other_ns / info["calls"] / 1e6,
       "hipevents_other_ms_per_call": info["stage_ms_per_call"]["other"],
       "rocprof_gemm_tflops": info["gemm_flops_per_call"] / (per_call * 1e-3) / 1e12,
       "hipevents_gemm_tflops": info["gemm_tflops"], "frames_per_call": info["frames_per_call"]}
print(json.dumps(res))
