"""Time the DWPose keypoint extractor (RTMPose-l whole-body, random weights) on cuda:0: frames/s and the
implicit-GEMM conv rate from per-launch hipEvents (vge_dwpose_profile_*).
python tools/time_dwpose.py [--frames 256] [--iters 5] [--persons 1]"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "video-gen-evals_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from vge import dwpose as D, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=256)
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--persons", type=int, default=0, help="persons per frame (0 = whole-frame box)")
ap.add_argument("--detector", action="store_true", help="also time the YOLOX-L detector on the same frames")
ap.add_argument("--chunk", type=int, default=64)
a = ap.parse_args()
cfg = D.RTMPOSE_L
t0 = time.time()
ex = D.DwposeExtractor(synth.make_rtmpose_state_dict(cfg), cfg, device="cuda:0", max_instances=2 * a.frames)
setup = time.time() - t0
frames = torch.from_numpy(synth.make_frames(3, a.frames)).cuda()
P = max(a.persons, 1)
boxes = np.tile(np.array([[20, 10, 230, 250]], np.float32), (a.frames, P, 1))
npers = np.full(a.frames, a.persons, np.int32)
ex.keypoints(frames, boxes, npers)
torch.cuda.synchronize()
ex.profile_begin(a.iters)
t = time.perf_counter()
for _ in range(a.iters):
    out = ex.keypoints(frames, boxes, npers)
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / a.iters
st, n, fl = ex.profile_read()
inst = ex.instances(npers)
print(json.dumps({"frames": a.frames, "instances": inst, "ms_per_call": dt * 1e3, "frames_per_s": a.frames / dt,
                  "stage_ms": {k: v / n for k, v in st.items()},
                  "gemm_tflops": fl / (st["gemm"] / n * 1e-3) / 1e12, "gflop_per_instance": fl / inst / 1e9,
                  "setup_s": setup, "finite": bool(torch.isfinite(out).all())}))
if a.detector:
    det = D.YoloxDetector(synth.make_yolox_state_dict(D.YOLOX_L), D.YOLOX_L, device="cuda:0", chunk=a.chunk)
    det.detect(frames)
    torch.cuda.synchronize()
    det.profile_begin(a.iters)
    t = time.perf_counter()
    for _ in range(a.iters):
        b, n = det.detect(frames)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / a.iters
    st, nc, fl = det.profile_read()
    print(json.dumps({"detector": "yolox_l", "frames": a.frames, "chunk": a.chunk, "ms_per_call": dt * 1e3,
                      "frames_per_s": a.frames / dt, "stage_ms": {k: v / nc for k, v in st.items()},
                      "gemm_tflops": fl / (st["gemm"] / nc * 1e-3) / 1e12, "gflop_per_frame": fl / a.frames / 1e9,
                      "persons": np.bincount(n.cpu().numpy(), minlength=3).tolist()}))
