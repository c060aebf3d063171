"""Calibrate the e2e chain's gate-detector weights (vge.synth.make_gate_frcnn_state_dict) on the GPU.

With classes 1..79 at -20, a proposal's person score is sigmoid(d - t), d = person logit - background logit (background
bias 0) and t the background bias.  The gate's count at bias t is the number of greedy-NMS (IoU 0.5) survivors among
the class-0 boxes with d > t: a survivor's status depends only on higher-scored boxes, so survivors of the NMS over
every proposal in d order answer every t at once.  A frame has exactly one person iff d_1 <= t < d_0 (its first two
survivors).  The tool reads the head / proposal taps of one detector pass with t = 0, picks the t that maximises the
fraction of pool frames with exactly one person (the middle of the best run, a margin against bf16 rounding), then
re-runs the detector with that bias and reports the measured fraction.
Usage (GPU box): python tools/frcnn_gate_calib.py [pool_frames]  -> gpurun_out/frcnn_gate_calib.json
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "video-gen-evals_amd"))
from vge import synth  # noqa: E402
from vge.frcnn import FRCNN_X101, FrcnnDetector  # noqa: E402


def nms_order(boxes, thr=0.5):
    """Greedy NMS survivors of boxes already sorted by score (IoU > thr suppresses)."""
    keep = []
    area = (boxes[:, 2] - boxes[:, 0]) * (boxes[:, 3] - boxes[:, 1])
    sup = np.zeros(len(boxes), bool)
    for i in range(len(boxes)):
        if sup[i]:
            continue
        keep.append(i)
        if len(keep) == 2:
            break
        xx1 = np.maximum(boxes[i, 0], boxes[:, 0])
        yy1 = np.maximum(boxes[i, 1], boxes[:, 1])
        xx2 = np.minimum(boxes[i, 2], boxes[:, 2])
        yy2 = np.minimum(boxes[i, 3], boxes[:, 3])
        inter = np.clip(xx2 - xx1, 0, None) * np.clip(yy2 - yy1, 0, None)
        sup |= inter / (area[i] + area - inter) > thr
    return keep


def decode(prop, d, size):
    w, h = prop[:, 2] - prop[:, 0], prop[:, 3] - prop[:, 1]
    cx, cy = prop[:, 0] + 0.5 * w, prop[:, 1] + 0.5 * h
    dx, dy = d[:, 0] / 10, d[:, 1] / 10
    dw, dh = np.minimum(d[:, 2] / 5, np.log(1000 / 16)), np.minimum(d[:, 3] / 5, np.log(1000 / 16))
    pcx, pcy, pw, ph = dx * w + cx, dy * h + cy, np.exp(dw) * w, np.exp(dh) * h
    b = np.stack([pcx - pw / 2, pcy - ph / 2, pcx + pw / 2, pcy + ph / 2], 1)
    return np.stack([np.clip(b[:, 0], 0, size[1]), np.clip(b[:, 1], 0, size[0]), np.clip(b[:, 2], 0, size[1]),
                     np.clip(b[:, 3], 0, size[0])], 1)


def run(bg, pool, taps=False):
    cfg = FRCNN_X101
    det = FrcnnDetector(synth.make_gate_frcnn_state_dict(cfg, bg=bg), cfg, device="cuda", chunk=32)
    out_n, pairs = [], []
    for f0 in range(0, pool.shape[0], 32):
        fr = pool[f0:f0 + 32]
        tp = None
        if taps:
            full = det.make_taps(fr.shape[0], 256, 256)
            tp = {k: full[k] for k in ("proposals", "n_proposals", "head")}
        o = det.detect(fr, taps=tp)
        out_n.append(o["n_person"].cpu().numpy())
        if taps:
            K = cfg.num_classes
            size = det.shapes(256, 256)["resized"]
            hd, pr, npr = tp["head"].cpu().numpy(), tp["proposals"].cpu().numpy(), tp["n_proposals"].cpu().numpy()
            for f in range(fr.shape[0]):
                n = int(npr[f])
                dd = hd[f, :n, 0] - hd[f, :n, K]
                order = np.argsort(-dd, kind="stable")
                bx = decode(pr[f, :n, :4][order], hd[f, :n, K + 1:K + 5][order], size)
                k = nms_order(bx)
                pairs.append((dd[order][k[0]] if k else -np.inf, dd[order][k[1]] if len(k) > 1 else -np.inf))
    det.close()
    return np.concatenate(out_n), np.asarray(pairs)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    pool = torch.from_numpy(synth.make_frame_pool(7000, n)).cuda()
    _, pairs = run(0.0, pool, taps=True)
    d0, d1 = pairs[:, 0], pairs[:, 1]
    cand = np.unique(np.concatenate([d0[np.isfinite(d0)], d1[np.isfinite(d1)]]))
    frac = np.array([np.mean((d1 <= t) & (t < d0)) for t in cand])
    i = int(np.argmax(frac))
    j = i
    while j + 1 < len(cand) and frac[j + 1] == frac[i]:
        j += 1
    t = float(0.5 * (cand[i] + cand[min(j + 1, len(cand) - 1)]))
    npers, _ = run(t, pool)
    res = {"pool_frames": n, "background_bias": t, "predicted_single_fraction": float(frac[i]),
           "measured_single_fraction": float(np.mean(npers == 1)),
           "person_count_histogram": np.bincount(np.minimum(npers, 5), minlength=6).tolist(),
           "d0_quantiles": np.quantile(d0[np.isfinite(d0)], [0, .1, .5, .9, 1]).tolist(),
           "d1_quantiles": np.quantile(d1[np.isfinite(d1)], [0, .1, .5, .9, 1]).tolist()}
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/frcnn_gate_calib.json", "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
