"""Time the TokenHMR extractor (full ViT-H/16 config, random weights) on cuda:0: frames/s and the backbone GEMM
rate from per-launch hipEvents (vge_hmr_profile_*).  python tools/time_hmr.py [--frames 256] [--iters 5]"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "video-gen-evals_amd"))
import torch  # noqa: E402

from vge import hmr as H, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=256)
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--depth", type=int, default=32)
a = ap.parse_args()
cfg = H.HmrConfig(depth=a.depth)
t0 = time.time()
sd = synth.make_hmr_state_dict(cfg)
ex = H.HmrExtractor(sd, cfg, device="cuda:0", max_frames=a.frames)
del sd
setup = time.time() - t0
frames = torch.from_numpy(synth.make_frames(3, a.frames)).cuda()
ex.extract(frames)
torch.cuda.synchronize()
ex.profile_begin(a.iters)
t = time.perf_counter()
for _ in range(a.iters):
    out = ex.extract(frames)
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / a.iters
st, n, fl = ex.profile_read()
gemm_ms = st["gemm"] / n
print(json.dumps({"frames": a.frames, "depth": a.depth, "ms_per_call": dt * 1e3, "frames_per_s": a.frames / dt,
                  "stage_ms": {k: v / n for k, v in st.items()},
                  "gemm_tflops": fl * a.frames / (gemm_ms * 1e-3) / 1e12, "setup_s": setup,
                  "finite": bool(torch.isfinite(out["vit"]).all())}))
