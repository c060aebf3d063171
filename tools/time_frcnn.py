"""Throughput of the gate detector (vge.frcnn.FrcnnDetector, full X101-32x8d-FPN at 800 px) on the GPU.

One warm pass (the conv tuner measures each layer shape there), then `passes` timed passes over `frames` synthetic
256 x 256 frames in chunks; hipEvents around each pass and the detector's per-stage profile (backbone GEMMs, head GEMMs,
everything else) -> frames/s and TFLOP/s of the two GEMM stages against the algorithmic FLOPs (grouped convolutions at
their grouped size).  Usage: python tools/time_frcnn.py [frames] [chunk] [passes] -> JSON line (+ gpurun_out/).
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "video-gen-evals_amd"))
from vge import synth  # noqa: E402
from vge.frcnn import FRCNN_X101, FrcnnDetector  # noqa: E402


def main():
    nf = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    passes = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    det = FrcnnDetector(synth.make_gate_frcnn_state_dict(FRCNN_X101), FRCNN_X101, device="cuda", chunk=chunk)
    frames = torch.from_numpy(synth.make_frame_pool(4242, nf)).cuda()
    t0 = time.perf_counter()
    det.detect(frames)
    torch.cuda.synchronize()
    warm = time.perf_counter() - t0
    det.profile_begin(passes)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(passes):
        o = det.detect(frames)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / passes
    stage, n, fl = det.profile_read()
    bb, hd = det.flops(256, 256)
    res = {"frames": nf, "chunk": chunk, "passes": passes, "ms_per_pass": ms, "frames_per_s": nf / ms * 1e3,
           "warm_pass_s": warm, "stage_ms_per_pass": {k: v / max(n, 1) for k, v in stage.items()},
           "gflop_per_frame": {"backbone_fpn_rpn": bb / 1e9, "box_head": hd / 1e9},
           "library_gemm_gflop_per_pass": [x / 1e9 for x in fl],
           "backbone_tflops": bb * nf / (stage["backbone_gemm"] / max(n, 1)) / 1e9,
           "head_tflops": hd * nf / (stage["head_gemm"] / max(n, 1)) / 1e9,
           "persons_per_frame_hist": torch.bincount(o["n_person"].clamp(max=5).cpu(), minlength=6).tolist()}
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/time_frcnn.json", "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
