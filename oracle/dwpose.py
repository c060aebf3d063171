"""ORACLE (test infrastructure only): torch CPU restatement of the DWPose whole-body keypoint extractor.

The reference runs DWPose per frame in modifications/process_video.py:59-91 (``pose(frame)`` ->
``flatten_first_person_no_padding(bodies, hands)``, lines 23-57) through ``DWposeDetector``
(modifications/dwpose_init.py:37-69: Wholebody() -> candidate / W, H; subset < 0.3 -> -1; body = first 18
OpenPose points; hands = vstack(candidate[:, 92:113], candidate[:, 113:])).  ``Wholebody`` and its models are
third-party code NOT in /root/reference (ControlNet's annotator/dwpose: wholebody.py, onnxdet.py, onnxpose.py;
models yolox_l.onnx and dw-ll_ucoco_384.onnx = RTMPose-l whole-body, downloaded at run time, no pinned
version), so this file restates their published algorithms:

  onnxpose.preprocess     bbox_xyxy2cs(padding 1.25), _fix_aspect_ratio(288/384), get_warp_matrix (rot 0) +
                          cv2.warpAffine(INTER_LINEAR, border 0) to 288x384 (uint8 result), (x - mean) / std on
                          the BGR channels; no detection -> the whole frame is the box
  RTMPose-l (mmpose)      CSPNeXt-P5 (stem 3x ConvModule, 4 stages of 3x3/s2 ConvModule [+ SPPBottleneck 5/9/13]
                          + CSPLayer(CSPNeXtBlock: 3x3 ConvModule, 5x5 depthwise + 1x1 ConvModule, identity
                          add; ChannelAttention = avgpool -> 1x1 conv -> hardsigmoid -> scale), BN + SiLU)
                          -> RTMCCHead (7x7 conv, flatten, ScaleNorm, Linear -> 256, RTMCCBlock gated attention
                          unit (ScaleNorm, uv Linear + SiLU, q/k = base * gamma + beta, relu(qk / sqrt(s))^2,
                          u * (kernel @ v), o Linear, res_scale shortcut), cls_x / cls_y Linears)
  onnxpose.postprocess    get_simcc_maximum (argmax, vals = min of the x / y maxima, locs = -1 where vals <= 0),
                          / split ratio, / input size * scale + center - scale / 2 (float64)
  wholebody.__call__      neck = mean of the shoulders (score = both > 0.3), insert at 17, mmpose -> openpose
                          reorder of the body points

Parity vs the upstream ONNX models is UNPINNED (no weights offline, nothing in the reference fixes these
numbers; cv2's fixed-point bilinear is restated in float).  With ``bf16=True`` the restatement rounds to
bfloat16 exactly where libvge's kernels store bf16 (conv / Linear operands and activations), so the GPU path
is compared against the same arithmetic up to f32 summation order.
"""
from __future__ import annotations

import math
from typing import Dict, Sequence

import numpy as np
import torch
import torch.nn.functional as F

BN_EPS = 1e-5  # mmpose RTMPose configs: norm_cfg SyncBN (default eps)
MEAN_BGR = (123.675, 116.28, 103.53)
STD_BGR = (58.395, 57.12, 57.375)
OPENPOSE18_FROM_WB = (0, 17, 6, 8, 10, 5, 7, 9, 12, 14, 16, 11, 13, 15, 2, 1, 4, 3)


def fold_bn(p: Dict[str, torch.Tensor], prefix: str, eps: float = BN_EPS):
    """ConvModule conv (no bias) + BN -> (w * s, beta - mean * s), s = gamma / sqrt(var + eps), all f32."""
    w = p[prefix + ".conv.weight"]
    s = p[prefix + ".bn.weight"] / torch.sqrt(p[prefix + ".bn.running_var"] + eps)
    return w * s.view(-1, 1, 1, 1), p[prefix + ".bn.bias"] - p[prefix + ".bn.running_mean"] * s


def affine_params(box, in_w: int, in_h: int):
    """(cx, cy, src_w, src_h) in float32 as libvge's host computes them (bbox_xyxy2cs + _fix_aspect_ratio)."""
    x0, y0, x1, y1 = (np.float32(v) for v in box)
    f = np.float32
    cx, cy = (x0 + x1) * f(0.5), (y0 + y1) * f(0.5)
    w, h = (x1 - x0) * f(1.25), (y1 - y0) * f(1.25)
    ar = f(in_w) / f(in_h)
    if w > h * ar:
        sw, sh = w, w / ar
    else:
        sw, sh = h * ar, h
    return cx, cy, sw, sh


def warp_input(frame_rgb: np.ndarray, box, in_w: int, in_h: int) -> np.ndarray:
    """cv2.warpAffine(INTER_LINEAR, BORDER_CONSTANT 0) of the BGR frame onto the in_h x in_w model input,
    restated in float32 with the kernel's operation order; uint8 result (round half to even), then
    normalised -> [3, in_h, in_w] float32 (BGR channel order, mean / std in that order)."""
    f = np.float32
    cx, cy, sw, sh = affine_params(box, in_w, in_h)
    k = sw / f(in_w)  # source pixels per model pixel
    H, W = frame_rgb.shape[:2]
    u = np.arange(in_w, dtype=np.float32)
    v = np.arange(in_h, dtype=np.float32)
    sx = cx + (u - f(0.5) * f(in_w)) * k
    sy = cy + (v - f(0.5) * f(in_h)) * k
    x0 = np.floor(sx)
    y0 = np.floor(sy)
    fx = (sx - x0).astype(np.float32)
    fy = (sy - y0).astype(np.float32)
    x0 = x0.astype(np.int64)
    y0 = y0.astype(np.int64)
    img = frame_rgb[..., ::-1].astype(np.float32)  # BGR

    def px(yy, xx):
        ok = (yy[:, None] >= 0) & (yy[:, None] < H) & (xx[None, :] >= 0) & (xx[None, :] < W)
        val = img[np.clip(yy, 0, H - 1)[:, None], np.clip(xx, 0, W - 1)[None, :]]
        return np.where(ok[..., None], val, f(0))

    p00, p01, p10, p11 = px(y0, x0), px(y0, x0 + 1), px(y0 + 1, x0), px(y0 + 1, x0 + 1)
    fx_, fy_ = fx[None, :, None], fy[:, None, None]
    top = (f(1) - fx_) * p00 + fx_ * p01
    bot = (f(1) - fx_) * p10 + fx_ * p11
    val = (f(1) - fy_) * top + fy_ * bot
    u8 = np.rint(np.clip(val, f(0), f(255))).astype(np.float32)
    mean = np.array(MEAN_BGR, np.float32)
    std = np.array(STD_BGR, np.float32)
    return ((u8 - mean) / std).transpose(2, 0, 1).astype(np.float32)


class OracleRtmpose:
    def __init__(self, sd: Dict[str, np.ndarray], cfg, bf16: bool = True):
        self.p = {k: torch.as_tensor(np.asarray(v, np.float32)) for k, v in sd.items()}
        self.c = cfg
        self.bf16 = bf16

    def r(self, x: torch.Tensor) -> torch.Tensor:  # a bf16 storage point of the GPU path
        return x.to(torch.bfloat16).float() if self.bf16 else x

    # ConvModule: conv + folded BN + SiLU (+ identity added after the activation, one rounding)
    def conv(self, x, prefix, stride=1, res=None, groups=1):
        w, b = fold_bn(self.p, prefix)
        k = w.shape[-1]
        if groups == 1:
            w = self.r(w)
        y = F.silu(F.conv2d(x, w, b, stride=stride, padding=k // 2, groups=groups))
        if res is not None:
            y = y + res
        return self.r(y)

    def channel_attention(self, x, prefix):
        a = x.mean(dim=(2, 3))
        a = a @ self.p[prefix + ".fc.weight"][:, :, 0, 0].t() + self.p[prefix + ".fc.bias"]
        a = F.hardsigmoid(a)
        return self.r(x * a[:, :, None, None])

    def csp(self, x, prefix, n, add_identity):
        short = self.conv(x, prefix + ".short_conv")
        main = self.conv(x, prefix + ".main_conv")
        for b in range(n):
            p = f"{prefix}.blocks.{b}"
            y = self.conv(main, p + ".conv1")
            y = self.conv(y, p + ".conv2.depthwise_conv", groups=y.shape[1])
            main = self.conv(y, p + ".conv2.pointwise_conv", res=main if add_identity else None)
        x = self.channel_attention(torch.cat([main, short], 1), prefix + ".attention")
        return self.conv(x, prefix + ".final_conv")

    def backbone(self, x):
        c = self.c
        x = self.r(x)
        x = self.conv(x, "backbone.stem.0", stride=2)
        x = self.conv(x, "backbone.stem.1")
        x = self.conv(x, "backbone.stem.2")
        for i, n in enumerate(c.stage_blocks):
            st = f"backbone.stage{i + 1}"
            x = self.conv(x, st + ".0", stride=2)
            j = 1
            if i == 3:
                y = self.conv(x, st + ".1.conv1")
                pools = [F.max_pool2d(y, k, stride=1, padding=k // 2) for k in (5, 9, 13)]
                x = self.conv(torch.cat([y] + pools, 1), st + ".1.conv2")
                j = 2
            x = self.csp(x, f"{st}.{j}", n, add_identity=(i < 3))
        return x

    @staticmethod
    def scale_norm(x, g, eps=1e-5):
        norm = torch.norm(x, dim=-1, keepdim=True) * (x.shape[-1] ** -0.5)
        return x / norm.clamp(min=eps) * g

    def head(self, feats):
        c, p = self.c, self.p
        y = F.conv2d(feats, self.r(p["head.final_layer.weight"]), p["head.final_layer.bias"],
                     padding=c.final_k // 2)
        N, K = y.shape[:2]
        y = y.flatten(2)                                            # [N, K, h*w]
        y = self.r(self.scale_norm(y, p["head.mlp.0.g"]))
        x = y @ self.r(p["head.mlp.1.weight"]).t()                  # [N, K, 256] f32
        # RTMCCBlock (self-attn, no rel bias / pos enc)
        xn = self.r(self.scale_norm(x, p["head.gau.ln.g"]))
        uv = F.silu(xn @ self.r(p["head.gau.uv.weight"]).t())
        E, S = c.gau_e, c.gau_s
        u, v, base = uv[..., :E], uv[..., E:2 * E], uv[..., 2 * E:]
        base = base.unsqueeze(2) * p["head.gau.gamma"][None, None] + p["head.gau.beta"]
        q, k = base[:, :, 0], base[:, :, 1]
        kern = torch.square(F.relu((q @ k.transpose(1, 2)) / math.sqrt(S)))
        o = self.r(u * (kern @ v))
        x = x * p["head.gau.res_scale.scale"] + o @ self.r(p["head.gau.o.weight"]).t()
        x = self.r(x)
        sx = x @ self.r(p["head.cls_x.weight"]).t()
        sy = x @ self.r(p["head.cls_y.weight"]).t()
        return sx, sy

    @torch.no_grad()
    def simcc(self, frames_rgb: np.ndarray, inst_frame: Sequence[int], inst_box) -> tuple:
        c = self.c
        x = np.stack([warp_input(frames_rgb[f], b, c.in_w, c.in_h) for f, b in zip(inst_frame, inst_box)])
        return self.head(self.backbone(torch.from_numpy(x)))

    @staticmethod
    def decode(sx: torch.Tensor, sy: torch.Tensor, split: int):
        """get_simcc_maximum + / split ratio -> locs [N, K, 2] float32 (model-input pixels), vals [N, K]."""
        xl = sx.argmax(-1)
        yl = sy.argmax(-1)
        mx, my = sx.amax(-1), sy.amax(-1)
        vals = torch.minimum(mx, my)
        locs = torch.stack([xl, yl], -1).float()
        locs[vals <= 0] = -1
        return locs / split, vals


def flatten_first_person(body: np.ndarray, hands):
    """process_video.py:23-57 flatten_first_person_no_padding restated: body = bodies['candidate'] [>= 18, 2],
    hands [2 * nums, 21, 2] (or [k, 2, 21, 2]) -> [120] (body 18 | hand_pair[0] | hand_pair[1]) or None."""
    if body is None or body.size == 0 or body.shape[0] < 18 or hands is None:
        return None
    h = np.asarray(hands)
    if h.ndim == 4:
        if h.shape[0] < 1 or h.shape[1:] != (2, 21, 2):
            return None
        pair = h[0]
    elif h.ndim == 3:
        if h.shape[0] < 2 or h.shape[1:] != (21, 2):
            return None
        pair = np.stack([h[0], h[1]], axis=0)
    else:
        return None
    return np.concatenate([body[:18].reshape(-1), pair[0].reshape(-1), pair[1].reshape(-1)], axis=0)


def wholebody_to_kp120(locs: np.ndarray, vals: np.ndarray, boxes, in_w: int, in_h: int, H: int, W: int) -> np.ndarray:
    """onnxpose.postprocess -> wholebody neck / OpenPose reorder -> dwpose_init.py:44-67 normalisation ->
    flatten_first_person (process_video.py:23-57), for ONE frame whose persons (detector order) are rows of
    locs / vals.  Float64 like numpy, cast to float32 at the end (np.asarray(video_kps, dtype=float32))."""
    P = locs.shape[0]
    cand = np.zeros((P, 134, 2))
    score = np.zeros((P, 134))
    for i in range(P):
        cx, cy, sw, sh = (float(v) for v in affine_params(boxes[i], in_w, in_h))
        kp = locs[i].astype(np.float64) / np.array([in_w, in_h]) * np.array([sw, sh]) + np.array([cx, cy]) \
            - np.array([sw, sh]) / 2
        sc = vals[i].astype(np.float64)
        neck = (kp[5] + kp[6]) / 2
        neck_s = float(sc[5] > 0.3 and sc[6] > 0.3)
        kpi = np.insert(kp, 17, neck, axis=0)
        sci = np.insert(sc, 17, neck_s)
        # wholebody reorder: new[openpose_idx] = new[mmpose_idx]
        op_idx = [1, 2, 3, 4, 6, 7, 8, 9, 10, 12, 13, 14, 15, 16, 17]
        mm_idx = [17, 6, 8, 10, 7, 9, 12, 14, 16, 13, 15, 2, 1, 4, 3]
        kpi[op_idx] = kpi[mm_idx]
        sci[op_idx] = sci[mm_idx]
        cand[i] = kpi
        score[i] = sci
    # DWposeDetector.__call__ (dwpose_init.py:44-67)
    cand[..., 0] /= float(W)
    cand[..., 1] /= float(H)
    body = cand[:, :18].copy().reshape(P * 18, 2)  # copied BEFORE the visibility mask: body points keep
    cand[score < 0.3] = -1                          # their coordinates whatever their score; hands get -1
    hands = np.vstack([cand[:, 92:113], cand[:, 113:]])
    return flatten_first_person(body, hands).astype(np.float32)
