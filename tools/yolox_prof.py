#!/usr/bin/env python3
"""The e2e bench's person detector alone (vge.synth.make_gate_detector_state_dict weights, 640x640 letterbox of 256x256
frames): hipEvents stage times per detect call, the same numbers bench_e2e reports as yolox_* (stage_ms, GEMM
TFLOP/s).  Run under `rocprofv3 --kernel-trace` and check with tools/yolox_prof_check.py: the conv kernels' summed
durations of the profiled calls against stage_ms["gemm"].

    python tools/yolox_prof.py [--frames 256] [--calls 3] [--chunk 64]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "video-gen-evals_amd"))
import torch  # noqa: E402

from vge import synth  # noqa: E402
from vge.dwpose import YOLOX_L, YoloxDetector  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=256)
ap.add_argument("--calls", type=int, default=3)
ap.add_argument("--chunk", type=int, default=64, help="frames per detector pass (vge_yolox_reserve)")
a = ap.parse_args()
det = YoloxDetector(synth.make_gate_detector_state_dict(YOLOX_L), YOLOX_L, device="cuda:0", chunk=a.chunk)
fr = torch.from_numpy(synth.make_frame_pool(5000, a.frames)).cuda()
for _ in range(2):  # the first call measures the per-layer conv variants (ConvTuner)
    det.detect(fr, with_scores=True)
torch.cuda.synchronize()
det.profile_begin(a.calls)
for _ in range(a.calls):
    det.detect(fr, with_scores=True)
torch.cuda.synchronize()
st, n, fl = det.profile_read()
out = {"frames_per_call": a.frames, "calls": n, "chunk": a.chunk, "chunks_per_call": -(-a.frames // a.chunk),
       "stage_ms_per_call": {k: v / n for k, v in st.items()}, "gemm_flops_per_call": fl,
       "gemm_tflops": fl / (st["gemm"] / n * 1e-3) / 1e12}
print(json.dumps(out))
