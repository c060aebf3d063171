#!/usr/bin/env python3
"""HBM traffic per frame of config 3's two GEMM engines from tools/profile_e2e.sh TAG (FETCH_SIZE x 2 + WRITE_SIZE, the
MI355X_MICROARCH.md HBM recipe, summed over dispatches):
  gemm_bf16_kernel  the TokenHMR ViT-H/16 backbone GEMMs (gemm_bf16_kernel and the hipBLASLt Cijk_ kernels), every
                    dispatch of tools/time_hmr.py's calls / its frames
  yolox_conv        the YOLOX-L detector's implicit-GEMM convs (and 1x1 convs the tuner put on gemm_bf16_kernel), the
                    dispatches of tools/yolox_prof.py's profiled calls (from the first of their letterbox_focus launches
                    on, in dispatch order) / their frames
  frcnn_conv        the Faster R-CNN gate detector's convs (backbone, FPN, RPN, box head: the implicit-GEMM kernels,
                    the 1x1 convs on gemm_bf16_kernel, the grouped 3x3 on gconv3_kernel, the fused stem + pool), the dispatches of
                    tools/time_frcnn.py's timed call (from its first frcnn_resize_h launch on) / its frames
-> profiles/pmc_e2e.json, keyed by the kernels' source hash (bench_e2e.py reports `traffic` only while it matches).
    python tools/pmc_e2e.py TAG"""
import collections
import csv
import glob
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402  (sources_sha: the hash bench_e2e.py checks)
from bench_e2e import E2E_KERNEL_SOURCES  # noqa: E402

tag = sys.argv[1]
OUT = ROOT / "gpurun_out"


def dispatches(name):
    """Dispatch_Id -> (kernel name, {counter: value summed over the dispatch's instances})"""
    per = {}
    for f in glob.glob(str(OUT / f"pe_{tag}_{name}" / "**" / "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k, d = per.setdefault(int(r["Dispatch_Id"]), (r["Kernel_Name"], collections.defaultdict(float)))
            d[r["Counter_Name"]] += float(r["Counter_Value"])
    return per


def last_json(log):
    return json.loads([ln for ln in open(OUT / log).read().splitlines() if ln.startswith("{")][-1])


def total(kind, keep):
    fe, wr = dispatches(f"{kind}_fetch"), dispatches(f"{kind}_write")
    ids = [i for i in sorted(fe) if keep(i, fe[i][0])]
    by = sum(fe[i][1]["FETCH_SIZE"] * 2 for i in ids) + sum(wr[i][1]["WRITE_SIZE"] for i in ids if i in wr)
    return by * 1024, len(ids)


hinfo = last_json(f"pe_{tag}_hmr_fetch.log")
h_frames = hinfo["frames"] * 3   # the warm call + 2 timed calls (tools/time_hmr.py --iters 2)
def lib_gemm(k):  # hipBLASLt (Tensile) GEMM kernels
    return k.startswith("Cijk_") or "Cijk_" in k[:40]


h_bytes, h_n = total("hmr", lambda i, k: "gemm_bf16_kernel" in k or lib_gemm(k))

yinfo = last_json(f"pe_{tag}_yolox_fetch.log")
fe = dispatches("yolox_fetch")
lb = [i for i in sorted(fe) if "letterbox_focus" in fe[i][0]]
first = lb[-yinfo["calls"] * yinfo["chunks_per_call"]]
def conv_like(k):
    return (("conv" in k and "bf16" in k) or "gemm_bf16_kernel" in k or "gconv3_kernel" in k or lib_gemm(k)
            or "frcnn_stem_pool" in k)


y_bytes, y_n = total("yolox", lambda i, k: i >= first and conv_like(k))
y_frames = yinfo["calls"] * yinfo["frames_per_call"]

finfo = last_json(f"pe_{tag}_frcnn_fetch.log")
fe = dispatches("frcnn_fetch")
rz = [i for i in sorted(fe) if "frcnn_resize_h" in fe[i][0]]
chunks = -(-finfo["frames"] // finfo["chunk"])
ffirst = rz[-finfo["passes"] * chunks]
f_bytes, f_n = total("frcnn", lambda i, k: i >= ffirst and conv_like(k))
f_frames = finfo["passes"] * finfo["frames"]

res = {"gemm_bf16_kernel": {"what": "TokenHMR ViT-H/16 backbone GEMMs (gemm_bf16_kernel + hipBLASLt)", "dispatches": h_n, "frames": h_frames,
                            "hbm_bytes_per_frame": h_bytes / h_frames,
                            "source_sha": bench.sources_sha(E2E_KERNEL_SOURCES["gemm_bf16_kernel"]),
                            "source": f"gpurun_out/pe_{tag}_hmr_*/ (tools/profile_e2e.sh {tag})"},
       "yolox_conv": {"what": "YOLOX-L convs (conv_bf16 / conv2 / conv2p, 1x1 on gemm_bf16)", "dispatches": y_n,
                      "frames": y_frames, "chunk": yinfo["chunk"], "hbm_bytes_per_frame": y_bytes / y_frames,
                      "source_sha": bench.sources_sha(E2E_KERNEL_SOURCES["yolox_conv"]),
                      "source": f"gpurun_out/pe_{tag}_yolox_*/ (tools/profile_e2e.sh {tag})"},
       "frcnn_conv": {"what": "Faster R-CNN X101-32x8d-FPN convs (backbone, FPN, RPN, box head: implicit GEMM, 1x1 on hipBLASLt, grouped 3x3 on gconv3)",
                      "dispatches": f_n, "frames": f_frames, "chunk": finfo["chunk"],
                      "hbm_bytes_per_frame": f_bytes / f_frames,
                      "source_sha": bench.sources_sha(E2E_KERNEL_SOURCES["frcnn_conv"]),
                      "source": f"gpurun_out/pe_{tag}_frcnn_*/ (tools/profile_e2e.sh {tag})"}}
(ROOT / "profiles" / "pmc_e2e.json").write_text(json.dumps(res, indent=1) + "\n")
print(json.dumps(res, indent=1))
