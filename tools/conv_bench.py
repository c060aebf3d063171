"""Time conv_bf16 (the DWPose / YOLOX implicit-GEMM conv) on representative layer shapes: v2 (256-row tiles, default
for Cout % 256 == 0; persistent grid) vs v2_one_tile (VGE_CONV_PERSIST=0) vs v1 (128-row tiles) vs v1_tall (256-row)
vs v2p_512x128 (variant 6, Cout <= 128) vs torch/MIOpen conv2d (bf16, channels_last).  python tools/conv_bench.py"""
import ctypes as C
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "video-gen-evals_amd"))
import torch  # noqa: E402

from vge import dwpose as D, lib as L  # noqa: E402

SHAPES = [  # name, n, H, W, Cin, Cout, k, stride[, residual]
    ("yolox_head0_fused_3x3", 64, 80, 80, 256, 512, 3, 1),
    ("yolox_dark3_bneck_3x3", 64, 80, 80, 128, 128, 3, 1),
    ("yolox_dark3_bneck_3x3_res", 64, 80, 80, 128, 128, 3, 1, True),
    ("yolox_dark2_bneck_3x3_res", 64, 160, 160, 64, 64, 3, 1, True),
    ("yolox_dark2_3x3_64_128", 64, 160, 160, 64, 128, 3, 2),
    ("yolox_1x1_128_128_80", 64, 80, 80, 128, 128, 1, 1),
    ("yolox_1x1_128_128_160", 64, 160, 160, 128, 128, 1, 1),
    ("yolox_1x1_64_64_160", 64, 160, 160, 64, 64, 1, 1),
    ("yolox_dark4_bneck_3x3", 64, 40, 40, 256, 256, 3, 1),
    ("yolox_dark3_down_3x3s2", 64, 160, 160, 128, 256, 3, 2),
    ("yolox_1x1_256_128", 64, 80, 80, 256, 128, 1, 1),
    ("yolox_1x1_256_256", 64, 80, 80, 256, 256, 1, 1),
    ("yolox_1x1_512_256", 64, 40, 40, 512, 256, 1, 1),
    ("yolox_1x1_1024_512", 64, 20, 20, 1024, 512, 1, 1),
    ("yolox_head_1x1_256", 64, 80, 80, 256, 256, 1, 1),
    ("rtm_stage1_3x3_64", 256, 96, 72, 64, 64, 3, 1),
    ("rtm_stem2_3x3_32_64", 256, 192, 144, 32, 64, 3, 1),
    ("rtm_final_7x7", 256, 12, 9, 1024, 133, 7, 1),
]


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


import argparse  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n-scale", type=int, default=1, help="multiply every shape's image count")
ap.add_argument("--match", default="", help="only shapes whose name contains this")
args = ap.parse_args()
lib = L.load()
lib.vge_debug_set_conv_v1.argtypes = [C.c_int]
lib.vge_debug_set_conv_persist.argtypes = [C.c_int]
lib.vge_debug_set_conv_tall.argtypes = [C.c_int]
lib.vge_debug_set_conv_variant.argtypes = [C.c_int]
res = []
def _bf_like(t):
    return torch.randn(t.shape, device=t.device).to(torch.bfloat16)


for name, n, H, W, Cin, Cout, k, st, *opt in SHAPES:
    if args.match not in name:
        continue
    n *= args.n_scale
    resid = bool(opt and opt[0])
    x = torch.randn(n, H, W, Cin, device="cuda").to(torch.bfloat16)
    w = (torch.randn(Cout, Cin, k, k, device="cuda") * (2.0 / (Cin * k * k)) ** 0.5)
    b = torch.zeros(Cout, device="cuda")
    Ho, Wo = (H + 2 * (k // 2) - k) // st + 1, (W + 2 * (k // 2) - k) // st + 1
    out_f32 = Cout % 8 != 0
    out = torch.empty(n, Ho, Wo, Cout, device="cuda", dtype=torch.float32 if out_f32 else torch.bfloat16)
    fl = 2.0 * n * Ho * Wo * Cout * Cin * k * k
    r = {"shape": name, "n": n, "gflop": fl / 1e9}
    rr = _bf_like(out) if resid and not out_f32 else None
    for name_v, v1, pers, tall, force in (("v2", 0, 1, 0, 0), ("v2_one_tile", 0, 0, 0, 0), ("v1", 1, 1, 0, 0),
                                          ("v1_tall", 1, 1, 1, 0), ("v2p_512x128", 0, 1, 0, 6)):
        if force == 6 and Cout > 128:
            continue
        lib.vge_debug_set_conv_v1(v1)
        lib.vge_debug_set_conv_persist(pers)
        lib.vge_debug_set_conv_tall(tall)
        lib.vge_debug_set_conv_variant(force)
        ms = timeit(lambda: D.conv_bf16(x, w, b, stride=st, pad=k // 2, act="none" if out_f32 else "silu",
                                        out_f32=out_f32, out=out, res=rr))
        r[name_v] = {"ms": ms, "tflops": fl / ms / 1e9}
    lib.vge_debug_set_conv_v1(0)
    lib.vge_debug_set_conv_persist(1)
    lib.vge_debug_set_conv_tall(0)
    lib.vge_debug_set_conv_variant(0)
    xc = x.permute(0, 3, 1, 2)  # NCHW view of NHWC memory = channels_last
    wc = w.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    try:
        ms = timeit(lambda: torch.nn.functional.conv2d(xc, wc, None, st, k // 2))
        r["miopen"] = {"ms": ms, "tflops": fl / ms / 1e9}
    except Exception as e:  # noqa: BLE001
        r["miopen"] = str(e)[:80]
    print(json.dumps(r), flush=True)
