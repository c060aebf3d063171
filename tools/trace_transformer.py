#!/usr/bin/env python3
"""Per-segment timeline of transformer_x3_kernel from a VGE_TRACE build (s_memtime stamps of every wave of
blocks 0..63; timing-only, built by tools/ablate.sh):

    VGE_LIB=.../build/trace/libvge.so python tools/trace_transformer.py [--windows 256]

Segments: 0 tokens, then per layer q, k, v, out, (ffn1_c, ffn2_c) x 4.  For each: mean cycles of the weight
stream ("stream") and of the epilogue up to the next segment's start ("epi"), wave 0 of each block.
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
ap.add_argument("--tx-w", type=int, default=0, help="windows per workgroup (vge_debug_set_tx_windows; 0 = automatic)")
a = ap.parse_args()
dev = torch.device("cuda", 0)
sd = synth.make_state_dict(synth.DIMS_RAW, synth.DIMS_DIFF)
enc = ops.Encoder(sd, device=dev, compute=a.compute)
x = torch.randn(a.windows, 32, 2596, device=dev)
enc.reserve(a.windows)
lib.load().vge_debug_set_tx_windows(a.tx_w)
for _ in range(3):
    enc.encode(x)
torch.cuda.synchronize()
L = lib.load()
buf = (C.c_longlong * (64 * 4 * 128))()
assert L.vge_debug_tx_trace(buf, 64 * 4 * 128) == 0
t = np.array(buf, dtype=np.int64).reshape(64, 4, 128)
names = ["tokens"]
for l in range(4):
    names += [f"L{l}_q", f"L{l}_k", f"L{l}_v", f"L{l}_out"]
    for c in range(4):
        names += [f"L{l}_ffn1_{c}", f"L{l}_ffn2_{c}"]
nseg = len(names)
w0 = t[:, 0]
out = {"total": float((w0[:, 126] - w0[:, 124]).mean()), "staging": float((w0[:, 0] - w0[:, 124]).mean()),
       "outputs": float((w0[:, 126] - w0[:, 125]).mean())}
stream = w0[:, 1:2 * nseg:2] - w0[:, 0:2 * nseg:2]
nxt = np.concatenate([w0[:, 2:2 * nseg:2], w0[:, 125:126]], axis=1)
epi = nxt - w0[:, 1:2 * nseg:2]
out["stream_total"] = float(stream.sum(axis=1).mean())
out["epi_total"] = float(epi.sum(axis=1).mean())
out["segments"] = {n: [round(float(stream[:, k].mean())), round(float(epi[:, k].mean()))] for k, n in enumerate(names)}
for base, nm in ((100, "L0_out"), (110, "L0_ffn2_3")):
    st = w0[:, base + 1:base + 7]
    prev = w0[:, 2 * names.index(nm) + 1]
    marks = np.concatenate([prev[:, None], st], axis=1)
    out[nm + "_fine"] = [round(float(x)) for x in np.diff(marks, axis=1).mean(axis=0)]
out["start_skew"] = float((t[:, 0, 124].max() - t[:, 0, 124].min()))
print(json.dumps(out))
