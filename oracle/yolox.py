"""ORACLE (test infrastructure only): torch CPU restatement of DWPose's YOLOX-L person detector.

DWPose's Wholebody (called by modifications/dwpose_init.py:41 through ``self.pose_estimation(oriImg)``) runs
``inference_detector`` (ControlNet annotator/dwpose/onnxdet.py, NOT in /root/reference, model yolox_l.onnx
downloaded at run time, no pinned version) before the pose model.  Restated from the published YOLOX
(Megvii-BaseDetection/YOLOX: CSPDarknet + YOLOPAFPN + YOLOXHead, BaseConv = conv + BN(eps 1e-3) + SiLU) and
onnxdet.py:

  preprocess            r = min(640 / h, 640 / w); cv2.resize(INTER_LINEAR) to (int(w r), int(h r)) into the
                        top-left of a 114-filled 640 x 640 canvas, BGR, uint8 values, no normalisation
  Focus                 space-to-depth: cat(x[::2, ::2], x[1::2, ::2], x[::2, 1::2], x[1::2, 1::2])
  demo_postprocess      (reg_xy + grid) * stride, exp(reg_wh) * stride over strides 8 / 16 / 32
  boxes / scores        xyxy / r; score = sigmoid(obj) * sigmoid(cls)
  multiclass_nms        class-aware greedy NMS (IoU with the +1 pixel convention, keep if ovr <= 0.45) of the
                        candidates with score > 0.1; then keep class 0 with score > 0.3, in score order

Only class 0 can survive the final filter and NMS is class-aware, so only the person class is computed; a box
with score <= 0.3 can only suppress lower-scored boxes, which the filter drops anyway, and only persons 0 and 1
reach the keypoints.npy row (dwpose_init.py:61-64, process_video.py:44-51), so the restated NMS returns the
first two kept persons and min(count, 2).  Ties between equal scores take the lowest anchor index (numpy's
argsort order for ties is unspecified).  cv2's fixed-point bilinear is restated in float.  Parity vs the
upstream ONNX model is UNPINNED.  With ``bf16=True`` activations / weights round to bfloat16 where libvge stores
them.
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch
import torch.nn.functional as F

BN_EPS = 1e-3  # YOLOX init_yolo: BatchNorm eps 1e-3 at inference


def letterbox_focus(frame_rgb: np.ndarray, S: int) -> np.ndarray:
    """onnxdet.preprocess + Focus, with the kernel's float operation order -> [12, S/2, S/2] float32 (0..255)."""
    f = np.float32
    H, W = frame_rgb.shape[:2]
    r = min(S / H, S / W)
    rh, rw = int(H * r), int(W * r)
    ix, iy = f(W / rw), f(H / rh)
    img = frame_rgb[..., ::-1].astype(np.float32)

    def axis(n_out, inv, n_in):
        d = np.arange(n_out, dtype=np.float32)
        s = np.maximum((d + f(0.5)) * inv - f(0.5), f(0))
        i0 = np.floor(s).astype(np.int64)
        fr = (s - i0.astype(np.float32)).astype(np.float32)
        edge = i0 >= n_in - 1
        i0 = np.where(edge, n_in - 1, i0)
        fr = np.where(edge, f(0), fr).astype(np.float32)
        i1 = np.minimum(i0 + 1, n_in - 1)
        return i0, i1, fr

    x0, x1, fx = axis(rw, ix, W)
    y0, y1, fy = axis(rh, iy, H)
    fx_, fy_ = fx[None, :, None], fy[:, None, None]
    top = (f(1) - fx_) * img[y0][:, x0] + fx_ * img[y0][:, x1]
    bot = (f(1) - fx_) * img[y1][:, x0] + fx_ * img[y1][:, x1]
    res = np.rint(np.clip((f(1) - fy_) * top + fy_ * bot, f(0), f(255))).astype(np.float32)
    canvas = np.full((S, S, 3), 114, np.float32)
    canvas[:rh, :rw] = res
    x = canvas.transpose(2, 0, 1)
    return np.concatenate([x[:, ::2, ::2], x[:, 1::2, ::2], x[:, ::2, 1::2], x[:, 1::2, 1::2]], 0)


class OracleYolox:
    def __init__(self, sd: Dict[str, np.ndarray], cfg, bf16: bool = True):
        self.p = {k: torch.as_tensor(np.asarray(v, np.float32)) for k, v in sd.items()}
        self.c = cfg
        self.bf16 = bf16

    def r(self, x):
        return x.to(torch.bfloat16).float() if self.bf16 else x

    def base(self, x, prefix, stride=1, res=None):
        p = self.p
        w = p[prefix + ".conv.weight"]
        s = p[prefix + ".bn.weight"] / torch.sqrt(p[prefix + ".bn.running_var"] + BN_EPS)
        wf, bf = w * s.view(-1, 1, 1, 1), p[prefix + ".bn.bias"] - p[prefix + ".bn.running_mean"] * s
        y = F.silu(F.conv2d(x, self.r(wf), bf, stride=stride, padding=w.shape[-1] // 2))
        if res is not None:
            y = y + res
        return self.r(y)

    def csp(self, x, prefix, n, shortcut):
        x1 = self.base(x, prefix + ".conv1")
        x2 = self.base(x, prefix + ".conv2")
        for i in range(n):
            y = self.base(x1, f"{prefix}.m.{i}.conv1")
            x1 = self.base(y, f"{prefix}.m.{i}.conv2", res=x1 if shortcut else None)
        return self.base(torch.cat([x1, x2], 1), prefix + ".conv3")

    def forward(self, frames_rgb: np.ndarray):
        """-> per level (stride, [n, h*w, 6] = reg xywh, obj logit, cls-0 logit)."""
        c, p = self.c, self.p
        x = torch.from_numpy(np.stack([letterbox_focus(f, c.in_size) for f in frames_rgb]))
        bb, d = "backbone.backbone.", c.depth
        x = self.base(self.r(x), bb + "stem.conv")
        x = self.csp(self.base(x, bb + "dark2.0", 2), bb + "dark2.1", d, True)
        x2 = self.csp(self.base(x, bb + "dark3.0", 2), bb + "dark3.1", 3 * d, True)
        x1 = self.csp(self.base(x2, bb + "dark4.0", 2), bb + "dark4.1", 3 * d, True)
        y = self.base(self.base(x1, bb + "dark5.0", 2), bb + "dark5.1.conv1")
        y = self.base(torch.cat([y] + [F.max_pool2d(y, k, 1, k // 2) for k in (5, 9, 13)], 1), bb + "dark5.1.conv2")
        x0 = self.csp(y, bb + "dark5.2", d, False)
        fpn0 = self.base(x0, "backbone.lateral_conv0")
        f0 = self.csp(torch.cat([F.interpolate(fpn0, scale_factor=2, mode="nearest"), x1], 1), "backbone.C3_p4", d, False)
        fpn1 = self.base(f0, "backbone.reduce_conv1")
        pan2 = self.csp(torch.cat([F.interpolate(fpn1, scale_factor=2, mode="nearest"), x2], 1), "backbone.C3_p3", d,
                        False)
        pan1 = self.csp(torch.cat([self.base(pan2, "backbone.bu_conv2", 2), fpn1], 1), "backbone.C3_n3", d, False)
        pan0 = self.csp(torch.cat([self.base(pan1, "backbone.bu_conv1", 2), fpn0], 1), "backbone.C3_n4", d, False)
        outs = []
        for k, (feat, stride) in enumerate(((pan2, 8), (pan1, 16), (pan0, 32))):
            h = self.base(feat, f"head.stems.{k}")
            cf = self.base(self.base(h, f"head.cls_convs.{k}.0"), f"head.cls_convs.{k}.1")
            rf = self.base(self.base(h, f"head.reg_convs.{k}.0"), f"head.reg_convs.{k}.1")
            reg = F.conv2d(rf, self.r(p[f"head.reg_preds.{k}.weight"]), p[f"head.reg_preds.{k}.bias"])
            obj = F.conv2d(rf, self.r(p[f"head.obj_preds.{k}.weight"]), p[f"head.obj_preds.{k}.bias"])
            cls = F.conv2d(cf, self.r(p[f"head.cls_preds.{k}.weight"][:1]), p[f"head.cls_preds.{k}.bias"][:1])
            o = torch.cat([reg, obj, cls], 1).flatten(2).transpose(1, 2)
            outs.append((stride, o))
        return outs


def decode(outs, frame_hw, S: int):
    """demo_postprocess + xyxy / ratio + score, float32 like numpy (float64 intermediates rounded on assignment)
    -> boxes [n, A, 4] float32, scores [n, A] float32."""
    H, W = frame_hw
    ratio = np.float32(min(S / H, S / W))
    boxes, scores = [], []
    for stride, o in outs:
        o = o.numpy()
        g = S // stride
        gy, gx = np.divmod(np.arange(g * g), g)
        cx = ((o[..., 0].astype(np.float64) + gx) * stride).astype(np.float32)
        cy = ((o[..., 1].astype(np.float64) + gy) * stride).astype(np.float32)
        w = (np.exp(o[..., 2].astype(np.float32)).astype(np.float64) * stride).astype(np.float32)
        h = (np.exp(o[..., 3].astype(np.float32)).astype(np.float64) * stride).astype(np.float32)
        b = np.stack([cx - w / np.float32(2), cy - h / np.float32(2), cx + w / np.float32(2), cy + h / np.float32(2)], -1)
        boxes.append((b / ratio).astype(np.float32))
        sig = lambda v: (np.float32(1) / (np.float32(1) + np.exp(-v.astype(np.float32)))).astype(np.float32)
        scores.append((sig(o[..., 4]) * sig(o[..., 5])).astype(np.float32))
    return np.concatenate(boxes, 1), np.concatenate(scores, 1)


def iou_plus1(a, b) -> np.float32:
    """onnxdet.nms overlap (float32, +1 pixel convention)."""
    f = np.float32
    area_a = (a[2] - a[0] + f(1)) * (a[3] - a[1] + f(1))
    area_b = (b[2] - b[0] + f(1)) * (b[3] - b[1] + f(1))
    w = np.maximum(f(0), np.minimum(a[2], b[2]) - np.maximum(a[0], b[0]) + f(1))
    h = np.maximum(f(0), np.minimum(a[3], b[3]) - np.maximum(a[1], b[1]) + f(1))
    inter = w * h
    return inter / (area_a + area_b - inter)


def two_persons(boxes: np.ndarray, scores: np.ndarray, nms_thr=0.45, keep_thr=0.3):
    """Greedy class-aware NMS restricted to what reaches DWPose: (kept boxes [<=2, 4], min(count, 2))."""
    ok = scores > keep_thr
    if not ok.any():
        return np.zeros((0, 4), np.float32), 0
    s = np.where(ok, scores, -np.inf)
    i0 = int(np.argmax(s))  # first index among ties
    s2 = s.copy()
    s2[i0] = -np.inf
    sup = np.array([not (iou_plus1(boxes[i0], boxes[j]) <= np.float32(nms_thr)) if np.isfinite(s2[j]) else True
                    for j in range(len(s2))])
    s2[sup] = -np.inf
    if not np.isfinite(s2).any():
        return boxes[[i0]], 1
    i1 = int(np.argmax(s2))
    return boxes[[i0, i1]], 2
