#!/usr/bin/env python3
"""Time vge_encode's stages (hipEvents inside libvge) for a given libvge.so (env VGE_LIB) on random
z-scored input.  Used for A/B ablations of kernel variants in one process per variant.

    VGE_LIB=/path/libvge.so python tools/time_encoder.py [--windows 256] [--calls 20] [--compute f32x3]
"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "video-gen-evals_amd"))

import torch  # noqa: E402

from vge import ops, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--windows", type=int, default=256)
ap.add_argument("--calls", type=int, default=20)
ap.add_argument("--compute", default="f32x3")
ap.add_argument("--tag", default="")
a = ap.parse_args()
dev = torch.device("cuda", 0)
sd = synth.make_state_dict(synth.DIMS_RAW, synth.DIMS_DIFF)
enc = ops.Encoder(sd, device=dev, compute=a.compute)
x = torch.randn(a.windows, 32, 2596, device=dev)
enc.reserve(a.windows)
for _ in range(3):
    enc.encode(x)
torch.cuda.synchronize()
enc.profile_begin(a.calls)
for _ in range(a.calls):
    enc.encode(x)
torch.cuda.synchronize()
ms, n = enc.profile_read()
print(json.dumps({"tag": a.tag, "windows": a.windows, **{k: round(v / n, 4) for k, v in ms.items()}}))
