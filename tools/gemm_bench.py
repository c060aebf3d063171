"""Extractor GEMM rate on cuda:0 at the ViT-H shapes (random bf16 operands, interleaved rounds in one process),
next to torch.matmul (hipBLASLt) on the same operands as a library reference point.
python tools/gemm_bench.py [--frames 256] [--rounds 5]"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "video-gen-evals_amd"))
import torch  # noqa: E402

from vge import hmr as H  # noqa: E402
from vge import lib as L  # noqa: E402

so = L.load()

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=256)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--only", default="", help="one shape name (qkv/proj/fc1/fc2)")
ap.add_argument("--waves", default="w8,w4,lib", help="variants to run (w8s: 8 waves on 16x16x32)")
a = ap.parse_args()
M = a.frames * 192
shapes = {"qkv": (M, 3840, 1280, "bf16"), "proj": (M, 1280, 1280, "res_f32"), "fc1": (M, 5120, 1280, "gelu_bf16"),
          "fc2": (M, 1280, 5120, "res_f32")}
res = {}
g = torch.Generator(device="cuda").manual_seed(0)
for name, (m, n, k, epi) in shapes.items():
    if a.only and name != a.only:
        continue
    A = (torch.rand((m, k), device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    W = (torch.rand((n, k), device="cuda", generator=g) * 2 - 1).to(torch.bfloat16) * k ** -0.5
    bias = torch.zeros(n, device="cuda")
    r = torch.zeros((m, n), device="cuda") if epi == "res_f32" else None
    out = torch.empty((m, n), device="cuda", dtype=torch.float32 if epi == "res_f32" else torch.bfloat16)
    t = {w: [] for w in a.waves.split(",")}
    for _ in range(a.rounds + 1):
        for which in t:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if which != "lib":
                so.vge_debug_set_gemm_waves({"w8": 8, "w4": 4, "w8s": 16}[which])
            e0.record()
            if which != "lib":
                H.gemm_bf16(A, W, epi, bias=bias, res=r, out=out)
            else:
                torch.matmul(A, W.t())
            e1.record()
            torch.cuda.synchronize()
            t[which].append(e0.elapsed_time(e1))
    if "w8s" in t and "w8" in t:  # same operands through both MFMA shapes
        outs = []
        for nw in (8, 16):
            so.vge_debug_set_gemm_waves(nw)
            o = torch.empty_like(out)
            H.gemm_bf16(A, W, epi, bias=bias, res=r, out=o)
            outs.append(o.float())
        torch.cuda.synchronize()
        d = (outs[0] - outs[1]).abs()
        res.setdefault("_check", {})[name] = {"max_abs_diff_w8_w8s": float(d.max()),
                                              "max_abs_out": float(outs[0].abs().max())}
    fl = 2.0 * m * n * k
    res[name] = {"M": m, "N": n, "K": k, "epi": epi}
    for which, v in t.items():
        v = sorted(v[1:])
        res[name][which + "_ms_med"] = v[len(v) // 2]
        res[name][which + "_tflops"] = fl / v[len(v) // 2] / 1e9
    so.vge_debug_set_gemm_waves(8)
print(json.dumps(res, indent=1))
