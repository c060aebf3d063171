"""Calibrate the e2e bench's person-detector weights (vge.synth.make_gate_detector_state_dict) on the GPU.

Runs the detector with obj_shift 0 over make_frame_pool's frames, reads the scores of the first two persons NMS keeps
(vge_yolox_detect_scored), turns them back into objectness logits (the person class is saturated, so score =
sigmoid(objectness)), and picks the common logit shift t that maximises the fraction of frames with exactly one
person above 0.5 (l0 > t >= l1).  Then re-runs the detector with that shift and reports the measured fraction.
Usage (GPU box): python tools/yolox_gate_calib.py [pool_frames]  -> gpurun_out/yolox_gate_calib.json
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "video-gen-evals_amd"))
from vge import synth  # noqa: E402
from vge.dwpose import YOLOX_L, YoloxDetector  # noqa: E402
from vge.extract import single_person_mask  # noqa: E402


def scores_of(shift, pool):
    det = YoloxDetector(synth.make_gate_detector_state_dict(YOLOX_L, obj_shift=shift), YOLOX_L, device="cuda", chunk=64)
    out_b, out_s = [], []
    for f0 in range(0, pool.shape[0], 256):
        b, _, s = det.detect(pool[f0:f0 + 256], with_scores=True)
        out_b.append(b.cpu().numpy())
        out_s.append(s.cpu().numpy())
    det.close()
    return np.concatenate(out_b), np.concatenate(out_s)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    pool = torch.from_numpy(synth.make_frame_pool(7000, n)).cuda()
    boxes, s = scores_of(0.0, pool)
    with np.errstate(divide="ignore"):
        lg = np.log(s.astype(np.float64)) - np.log1p(-s.astype(np.float64))   # s = 0 (absent) -> -inf
    l0, l1 = lg[:, 0], lg[:, 1]
    cand = np.unique(np.concatenate([l0[np.isfinite(l0)], l1[np.isfinite(l1)]]))
    frac = np.array([np.mean((l0 > t) & ~(l1 > t)) for t in cand])
    i = int(np.argmax(frac))
    # the middle of the best run of thresholds (a margin against bf16 rounding differences between boxes)
    j = i
    while j + 1 < len(cand) and frac[j + 1] == frac[i]:
        j += 1
    t = float(0.5 * (cand[i] + cand[min(j + 1, len(cand) - 1)]))
    _, s2 = scores_of(t, pool)
    single = single_person_mask(s2)
    w = boxes[:, 0, 2] - boxes[:, 0, 0]
    h = boxes[:, 0, 3] - boxes[:, 0, 1]
    res = {"pool_frames": n, "obj_shift": t, "predicted_single_fraction": float(frac[i]),
           "measured_single_fraction": float(single.mean()),
           "l0_quantiles": np.quantile(l0[np.isfinite(l0)], [0, .1, .5, .9, 1]).tolist(),
           "l1_quantiles": np.quantile(l1[np.isfinite(l1)], [0, .1, .5, .9, 1]).tolist() if np.isfinite(l1).any() else None,
           "box0_w_quantiles": np.quantile(w, [0, .5, 1]).tolist(), "box0_h_quantiles": np.quantile(h, [0, .5, 1]).tolist(),
           "single_per_scene": single.reshape(-1, 4).sum(1).tolist()}
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/yolox_gate_calib.json", "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "single_per_scene"}))


if __name__ == "__main__":
    main()
