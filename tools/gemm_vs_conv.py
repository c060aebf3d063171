#!/usr/bin/env python3
"""The ViT-H GEMM shapes (K rounded to a power of two, as the conv path needs) through three kernels on the same bf16
operands: gemm_bf16_kernel (one 256 x 256 tile per workgroup, LDS epilogue), the implicit-GEMM conv as a 1x1 conv of
M one-pixel images (persistent conv2p_bf16_kernel 256 x 256, register epilogue: conv variant 3) and torch.matmul
(hipBLASLt).  Median of `--rounds` interleaved rounds, hipEvents.   python tools/gemm_vs_conv.py [--frames 256]"""
import argparse
import ctypes as C
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "video-gen-evals_amd"))
import torch  # noqa: E402

from vge import dwpose as D, hmr as H, lib as L  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=256)
ap.add_argument("--rounds", type=int, default=5)
a = ap.parse_args()
so = L.load()
so.vge_debug_set_conv_variant.argtypes = [C.c_int]
M = a.frames * 192
shapes = {"qkv": (3840, 1024), "proj": (1280, 1024), "fc1": (5120, 1024), "fc2": (1280, 4096)}
g = torch.Generator(device="cuda").manual_seed(0)
res = {}
for name, (N, K) in shapes.items():
    A = ((torch.rand((M, K), device="cuda", generator=g) * 2 - 1)).to(torch.bfloat16)
    W = ((torch.rand((N, K), device="cuda", generator=g) * 2 - 1) * K ** -0.5)
    Wb = W.to(torch.bfloat16)
    bias = torch.zeros(N, device="cuda")
    out = torch.empty((M, N), device="cuda", dtype=torch.bfloat16)
    x4 = A.view(M, 1, 1, K)
    w4 = W.view(N, K, 1, 1)
    wp = D.pack_conv_weight(w4)
    bp = torch.zeros(wp.shape[0], dtype=torch.float32, device="cuda")
    lib = D._sig(so)

    def conv(variant):
        so.vge_debug_set_conv_variant(variant)
        L.check(lib.vge_op_conv_bf16(D._ptr(x4), K, D._ptr(wp), D._ptr(bp), D._ptr(out), N, None, 0, None, M, 1, 1, K,
                                     1, 1, 1, 0, N, 0, 0, 0, D._stream(x4.device)), "conv")
        so.vge_debug_set_conv_variant(0)

    runs = {"gemm": lambda: H.gemm_bf16(A, Wb, "bf16", bias=bias, out=out), "conv2p": lambda: conv(3),
            "conv2_one_tile": lambda: conv(2), "lib": lambda: torch.matmul(A, Wb.t())}
    t = {k: [] for k in runs}
    for _ in range(a.rounds + 1):
        for k, fn in runs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            t[k].append(e0.elapsed_time(e1))
    fl = 2.0 * M * N * K
    res[name] = {"M": M, "N": N, "K": K}
    for k, v in t.items():
        v = sorted(v[1:])
        res[name][k + "_tflops"] = round(fl / v[len(v) // 2] / 1e9, 1)
    # same bytes out of the two of ours (bias 0, no activation): bit-identical GEMMs?
    H.gemm_bf16(A, Wb, "bf16", bias=bias, out=out)
    o1 = out.clone()
    conv(3)
    res[name]["gemm_vs_conv2p_max_abs"] = float((o1.float() - out.float()).abs().max())
print(json.dumps(res, indent=1))
