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
ap.add_argument("--waves", default="w8,w4,lib", help="variants to run (w8: 8 waves on 32x32x16, w8s: on 16x16x32, w2: gemm2, "
                                                     "auto: the default, p: the persistent kernel gemmp where it applies)")
a = ap.parse_args()
M = a.frames * 192
shapes = {"qkv": (M, 3840, 1280, "bf16"), "proj": (M, 1280, 1280, "res_f32"), "fc1": (M, 5120, 1280, "gelu_bf16"),
          "fc2": (M, 1280, 5120, "res_f32")}
NW = {"w8": 8, "w4": 4, "w8s": 16, "w2": 2, "auto": 1, "p": 1}
res = {}
g = torch.Generator(device="cuda").manual_seed(0)
for name, (m, n, k, epi) in shapes.items():
    if a.only and name != a.only:
        continue
    A = (torch.rand((m, k), device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    W = (torch.rand((n, k), device="cuda", generator=g) * 2 - 1).to(torch.bfloat16) * k ** -0.5
    bias = torch.rand(n, device="cuda", generator=g) * 0.2 - 0.1
    r = torch.randn((m, n), device="cuda", generator=g) * 0.5 if epi == "res_f32" else None
    out = torch.empty((m, n), device="cuda", dtype=torch.float32 if epi == "res_f32" else torch.bfloat16)
    t = {w: [] for w in a.waves.split(",")}
    for _ in range(a.rounds + 1):
        for which in t:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if which != "lib":
                so.vge_debug_set_gemm_waves(NW[which])
                so.vge_debug_set_gemm_persist(1 if which == "p" else 0)
            e0.record()
            if which != "lib":
                H.gemm_bf16(A, W, epi, bias=bias, res=r, out=out)
            else:
                torch.matmul(A, W.t())
            e1.record()
            torch.cuda.synchronize()
            t[which].append(e0.elapsed_time(e1))
    if "w8" in t:  # same operands through every variant: bitwise vs the 256 x 256 kernel on 32x32x16
        outs = {}
        for which in [w for w in t if w != "lib"]:
            so.vge_debug_set_gemm_waves(NW[which])
            so.vge_debug_set_gemm_persist(1 if which == "p" else 0)
            o = torch.empty_like(out)
            if r is not None:
                o2 = r.clone()
                H.gemm_bf16(A, W, epi, bias=bias, res=o2, out=o2)
                o = o2
            else:
                H.gemm_bf16(A, W, epi, bias=bias, res=r, out=o)
            outs[which] = o.float()
        torch.cuda.synchronize()
        for which, o in outs.items():
            if which != "w8":
                res.setdefault("_check", {}).setdefault(name, {})["max_abs_diff_w8_" + which] = float(
                    (outs["w8"] - o).abs().max())
        res["_check"][name]["max_abs_out"] = float(outs["w8"].abs().max())
    fl = 2.0 * m * n * k
    res[name] = {"M": m, "N": n, "K": k, "epi": epi}
    for which, v in t.items():
        v = sorted(v[1:])
        res[name][which + "_ms_med"] = v[len(v) // 2]
        res[name][which + "_tflops"] = fl / v[len(v) // 2] / 1e9
    so.vge_debug_set_gemm_waves(1)
    so.vge_debug_set_gemm_persist(0)
print(json.dumps(res, indent=1))
