#!/usr/bin/env python3
"""Precision / time of the f16 throughput mode per stage kept in 3xfp16 (VGE_F16_MIX bits: 1 stem, 2 transformer split, 4 transformer activations split)
against the oracle on bench.py's config-2 clips (256 windows, bench-like stats and centroids).

    python tools/f16_precision.py [--n 256]
"""
import argparse
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "video-gen-evals_amd"))
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=256)
a = ap.parse_args()
from tests.test_bench_parity import _oracle  # noqa: E402
from vge import ops  # noqa: E402

dev = "cuda:0"
o = _oracle(a.n)
feats = torch.from_numpy(o["feats"]).to(dev)
first = torch.arange(a.n + 1, dtype=torch.int32, device=dev)
vcls = o["vcls"].to(torch.int32).to(dev)
cent = o["cent"].to(dev)
for compute, mix in (("f32x3", 0), ("f16", 0), ("f16", 2), ("f16", 4), ("f16", 5), ("f16", 3)):
    os.environ["VGE_F16_MIX"] = str(mix)
    enc = ops.Encoder(o["sd"], device=dev, compute=compute)
    enc.reserve(a.n)
    for _ in range(3):
        seq, _, tcw = enc.encode(feats, frame_embed=False, tc=True)
    enc.profile_begin(10)
    for _ in range(10):
        seq, _, tcw = enc.encode(feats, frame_embed=False, tc=True)
    torch.cuda.synchronize()
    ms, nc = enc.profile_read()
    ac, tc = ops.score_videos(seq, tcw, first, vcls, cent)
    print(json.dumps({"compute": compute, "mix": mix, "seq": (seq.cpu() - o["seq"]).abs().max().item(),
                      "ac": (ac.cpu() - o["ac"]).abs().max().item(), "tc": (tc.cpu() - o["tc"]).abs().max().item(),
                      **{k: round(v / nc, 4) for k, v in ms.items()}}))
    del enc
