#!/usr/bin/env python3
"""Encode fixed random z-scored feats with the library at VGE_LIB (f32x3) and save seq / frame embeds / TC terms, for
comparing kernel variants bit for bit.  VGE_LIB=... python tools/enc_dump.py OUT.npz [--windows 256 600]"""
import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "video-gen-evals_amd"))
import torch  # noqa: E402

from vge import ops, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("out")
ap.add_argument("--windows", type=int, nargs="+", default=[256, 600, 37])
a = ap.parse_args()
dev = torch.device("cuda", 0)
enc = ops.Encoder(synth.make_state_dict(synth.DIMS_RAW, synth.DIMS_DIFF), device=dev, compute="f32x3")
res = {}
for n in a.windows:
    g = torch.Generator().manual_seed(n)
    x = torch.randn(n, 32, 2596, generator=g).to(dev)
    enc.reserve(n)
    s, f, t = enc.encode(x, frame_embed=True, tc=True)
    torch.cuda.synchronize()
    res[f"seq{n}"], res[f"fe{n}"], res[f"tc{n}"] = s.cpu().numpy(), f.cpu().numpy(), t.cpu().numpy()
np.savez(a.out, **res)
