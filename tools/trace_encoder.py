#!/usr/bin/env python3
"""Per-phase timeline of conv_encoder_x3_kernel from a VGE_TRACE build (s_memtime stamps of every wave of
blocks 0..63; timing-only, built by tools/ablate.sh):

    VGE_LIB=.../build/trace/libvge.so python tools/trace_encoder.py [--windows 256]

For each phase: mean cycles of wave 0 ("w0"), of the slowest wave ("max") and the spread between the first
and the last wave to reach the phase's end stamp ("skew").  Phases: stem staging, stem stream, stem
epilogue, 8 x (conv stream, conv epilogue [of which "gelu": stream end -> before the first reduction]),
proj stream, output store.
"""
import argparse
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "video-gen-evals_amd"))

import torch  # noqa: E402

from vge import lib, ops, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--windows", type=int, default=256)
ap.add_argument("--compute", default="f32x3")
a = ap.parse_args()
dev = torch.device("cuda", 0)
sd = synth.make_state_dict(synth.DIMS_RAW, synth.DIMS_DIFF)
enc = ops.Encoder(sd, device=dev, compute=a.compute)
x = torch.randn(a.windows, 32, 2596, device=dev)
enc.reserve(a.windows)
for _ in range(3):
    enc.encode(x)
torch.cuda.synchronize()
L = lib.load()
buf = (C.c_longlong * (64 * 8 * 32))()
assert L.vge_debug_x3_trace(buf, 64 * 8 * 32) == 0
t = np.array(buf, dtype=np.int64).reshape(64, 8, 32)
names = ["stem_stage", "stem_stream", "stem_epi"]
for k in range(8):
    names += [f"conv{k}_stream", f"conv{k}_epi"]
names += ["proj_stream", "out_store"]
out = {"blocks": 64, "encoders": np.bincount(t[:, 0, 31], minlength=10).tolist(),
       "total_cycles_w0": float((t[:, 0, 21] - t[:, 0, 0]).mean())}
for j, n in enumerate(names):
    d = t[:, :, j + 1] - t[:, :, j]
    out[n] = {"w0": round(float(d[:, 0].mean())), "max": round(float(d.max(axis=1).mean())),
              "skew": round(float((t[:, :, j + 1].max(axis=1) - t[:, :, j + 1].min(axis=1)).mean()))}
for k in range(8):
    g = t[:, :, 22 + k] - t[:, :, 4 + 2 * k]
    out[f"conv{k}_gelu"] = {"w0": round(float(g[:, 0].mean())), "max": round(float(g.max(axis=1).mean()))}
W = t[:, 0, 30]  # f16 unit kernel: windows of each block's unit (0 in the quad kernel's trace)
if W.any():
    out["unit_windows"] = {int(w): {"blocks": int((W == w).sum()),
                                    "total_cycles_w0": float((t[W == w, 0, 21] - t[W == w, 0, 0]).mean()),
                                    "conv_stream_w0": float(np.mean([(t[W == w, 0, 4 + 2 * k] - t[W == w, 0, 3 + 2 * k]
                                                                      if k else t[W == w, 0, 4] - t[W == w, 0, 3])
                                                                     for k in range(8)])),
                                    "conv_epi_w0": float(np.mean([t[W == w, 0, 5 + 2 * k] - t[W == w, 0, 4 + 2 * k]
                                                                  for k in range(8)]))}
                             for w in sorted(set(W.tolist()))}
print(json.dumps(out))
