"""Library reference points for the extractor GEMMs on cuda:0: our gemm_bf16_kernel (bias epilogue, bf16 out) next to
hipBLASLt through torch -- addmm (bias), _addmm_activation (bias + GELU / ReLU as a library epilogue) and matmul
without an epilogue -- at the ViT-H shapes (M = 49,152) and the gate detector's 1x1 conv shapes (128-frame chunk at
800 px), random bf16 operands, interleaved rounds, median ms.  A probe of what the library reaches on these shapes; it
is not on the product path.   python tools/lib_gemm_probe.py [--rounds 5] -> JSON"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "video-gen-evals_amd"))
import torch  # noqa: E402

from vge import hmr as H  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=5)
a = ap.parse_args()
SHAPES = {  # name: (M, N, K)
    "vit_qkv": (49152, 3840, 1280), "vit_fc1": (49152, 5120, 1280), "vit_fc2": (49152, 1280, 5120),
    "res2_conv1": (128 * 40000, 256, 256), "res3_conv1": (128 * 10000, 512, 512),
    "res4_conv1": (128 * 2500, 1024, 1024), "res4_conv3": (128 * 2500, 1024, 1024 // 2 * 2),
    "res5_conv1": (80128, 2048, 2048), "box_fc1": (128000, 1024, 12544),
}
g = torch.Generator(device="cuda").manual_seed(0)
res = {}
for name, (m, n, k) in SHAPES.items():
    A = (torch.rand((m, k), device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    W = ((torch.rand((n, k), device="cuda", generator=g) * 2 - 1) * k ** -0.5).to(torch.bfloat16)
    bias32 = torch.rand(n, device="cuda", generator=g) * 0.2 - 0.1
    bias16 = bias32.to(torch.bfloat16)
    out = torch.empty((m, n), device="cuda", dtype=torch.bfloat16)
    arms = {
        "ours_bias": lambda: H.gemm_bf16(A, W, "bf16", bias=bias32, out=out),
        "lib_matmul": lambda: torch.matmul(A, W.t()),
        "lib_addmm_bias": lambda: torch.addmm(bias16, A, W.t()),
        "lib_bias_relu": lambda: torch._addmm_activation(bias16, A, W.t(), use_gelu=False),
        "lib_bias_gelu": lambda: torch._addmm_activation(bias16, A, W.t(), use_gelu=True),
    }
    t = {k_: [] for k_ in arms}
    for _ in range(a.rounds + 1):
        for k_, f in arms.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f()
            e1.record()
            torch.cuda.synchronize()
            t[k_].append(e0.elapsed_time(e1))
    fl = 2.0 * m * n * k
    res[name] = {"M": m, "N": n, "K": k}
    for k_, v in t.items():
        v = sorted(v[1:])
        res[name][k_ + "_tflops"] = round(fl / v[len(v) // 2] / 1e9, 1)
    del A, W, out
    torch.cuda.empty_cache()
print(json.dumps(res, indent=1))
