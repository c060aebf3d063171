"""ORACLE (test infrastructure only): torch CPU restatement of TokenHMR's single-person gate detector.

The reference gates every frame on detectron2's COCO Faster R-CNN X101-32x8d-FPN (modifications/mesh_generator.py:69-73
builds ``DefaultPredictor`` from ``COCO-Detection/faster_rcnn_X_101_32x8d_FPN_3x.yaml`` with SCORE_THRESH_TEST 0.25;
mesh_generator.py:103-117 keeps a frame iff exactly one ``pred_classes == 0`` box has ``scores > 0.5``).  detectron2 is
third-party code absent from /root/reference (no pinned version; weights downloaded from the model zoo at run time),
so its published inference path is restated here:

  DefaultPredictor.__call__      BGR uint8 frame -> ResizeShortestEdge(800, 800, max 1333) (PIL Image.resize BILINEAR
                                 on uint8: fixed-point two-pass resample, restated bit-exactly by `resize_pil`) ->
                                 float32 CHW
  GeneralizedRCNN.preprocess     (x - PIXEL_MEAN) / PIXEL_STD (BGR 103.530 116.280 123.675 / 57.375 57.120 58.395),
                                 ImageList padded with 0 to a multiple of 32
  ResNeXt-101 32x8d (C2 model)   stem conv 7x7/2 + FrozenBN + ReLU, max_pool 3x3/2 pad 1; BottleneckBlocks (3, 4, 23,
                                 3), stride on the grouped 3x3 (STRIDE_IN_1X1 False), 32 groups, bottleneck width 256
                                 doubling per stage, shortcut 1x1 + FrozenBN on each stage's first block, relu(out +
                                 shortcut); FrozenBN eps 1e-5
  FPN                            lateral 1x1 + output 3x3 (bias, no norm), nearest 2x top-down sum, P6 =
                                 max_pool2d(P5, 1, 2)
  RPN                            StandardRPNHead (3x3 conv + ReLU, 1x1 objectness (3) and deltas (12)), anchors of
                                 sizes 32..512 x ratios (0.5, 1, 2), offset 0; per level top-1000 logits, decode
                                 (weights 1, clamp log(1000/16)), clip, nonempty, batched_nms 0.7 over levels, top 1000
  ROIPooler                      ROIAlignV2 7x7 (aligned, sampling_ratio 0 = adaptive), level = floor(4 + log2(sqrt(area)
                                 / 224 + 1e-8)) clamped to P2..P5
  FastRCNNConvFCHead / outputs   flatten -> fc1 1024 + ReLU -> fc2 1024 + ReLU -> cls_score (81) / bbox_pred (320);
                                 softmax, per-class decode (10, 10, 5, 5), clip, score > 0.25, batched_nms 0.5, top 100
  detector_postprocess           boxes scaled to the input frame size, clipped, nonempty

Conventions where the upstream result depends on the platform: ties between equal scores keep the lower index (stable
sorts); batched_nms uses torchvision's coordinate trick (boxes + class / level x (max coordinate + 1)), as on CUDA for
these sizes; every float expression is evaluated in float32 without fused multiply-adds; softmax = exp(x - max) / sum.
With ``bf16=True`` weights (after the FrozenBN fold) and activations round to bfloat16 exactly where libvge stores them.
Parity vs detectron2's own implementation and its trained weights is UNPINNED (absent offline); the resize is pinned
against Pillow itself (tests/test_frcnn_oracle.py).
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F

PIXEL_MEAN = (103.530, 116.280, 123.675)   # BGR, detectron2 defaults.py _C.MODEL.PIXEL_MEAN
PIXEL_STD = (57.375, 57.120, 58.395)       # faster_rcnn_X_101_32x8d_FPN_3x.yaml MODEL.PIXEL_STD
BN_EPS = 1e-5                              # FrozenBatchNorm2d
SCALE_CLAMP = math.log(1000.0 / 16)        # Box2BoxTransform scale_clamp
STAGE_BLOCKS = {50: (3, 4, 6, 3), 101: (3, 4, 23, 3), 152: (3, 8, 36, 3)}
PRECISION_BITS = 32 - 8 - 2                # Pillow Resample.c (8 bpc)

f32 = np.float32


# --------------------------------------------------------------------------------------------- preprocessing
def output_shape(h: int, w: int, short: int, max_size: int) -> Tuple[int, int]:
    """ResizeShortestEdge.get_output_shape."""
    size = short * 1.0
    scale = size / min(h, w)
    if h < w:
        newh, neww = size, scale * w
    else:
        newh, neww = scale * h, size
    if max(newh, neww) > max_size:
        scale = max_size * 1.0 / max(newh, neww)
        newh = newh * scale
        neww = neww * scale
    return int(newh + 0.5), int(neww + 0.5)


def pil_coeffs(in_size: int, out_size: int):
    """Pillow precompute_coeffs (bilinear, box = whole axis) + normalize_coeffs_8bpc -> (xmin [out], xmax [out],
    int32 coefficients [out, ksize])."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    kk = np.zeros((out_size, ksize), np.int64)
    xmin_a = np.zeros(out_size, np.int64)
    xmax_a = np.zeros(out_size, np.int64)
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = int(center - support + 0.5)
        xmin = max(xmin, 0)
        xmax = int(center + support + 0.5)
        xmax = min(xmax, in_size) - xmin
        ws = []
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            ws.append(1.0 - t if t < 1.0 else 0.0)
        ww = sum(ws)
        for x in range(xmax):
            w = ws[x] / ww if ww != 0.0 else ws[x]
            kk[xx, x] = int(-0.5 + w * (1 << PRECISION_BITS)) if w < 0 else int(0.5 + w * (1 << PRECISION_BITS))
        xmin_a[xx], xmax_a[xx] = xmin, xmax
    return xmin_a, xmax_a, kk


def _resample_axis(img: np.ndarray, axis: int, out_size: int) -> np.ndarray:
    xmin, xmax, kk = pil_coeffs(img.shape[axis], out_size)
    src = np.moveaxis(img.astype(np.int64), axis, 0)
    acc = np.full((out_size,) + src.shape[1:], 1 << (PRECISION_BITS - 1), np.int64)
    for k in range(kk.shape[1]):
        idx = np.minimum(xmin + k, src.shape[0] - 1)
        w = np.where(k < xmax, kk[:, k], 0).reshape((-1,) + (1,) * (src.ndim - 1))
        acc += src[idx] * w
    out = np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8)
    return np.moveaxis(out, 0, axis)


def resize_pil(img: np.ndarray, newh: int, neww: int) -> np.ndarray:
    """PIL Image.fromarray(img).resize((neww, newh), Image.BILINEAR) for uint8 [H, W, C]: the horizontal pass first,
    then the vertical one, each rounding to uint8 (Resample.c ImagingResampleInner); an axis whose size does not change
    is not resampled."""
    out = img
    if neww != img.shape[1]:
        out = _resample_axis(out, 1, neww)
    if newh != img.shape[0]:
        out = _resample_axis(out, 0, newh)
    return out


def preprocess(frame_rgb: np.ndarray, cfg) -> Tuple[np.ndarray, Tuple[int, int]]:
    """DefaultPredictor + preprocess_image for one RGB uint8 frame -> (normalised BGR float32 [3, Hp, Wp] zero-padded
    to a multiple of 32, (newh, neww))."""
    bgr = np.ascontiguousarray(frame_rgb[..., ::-1])
    h, w = bgr.shape[:2]
    nh, nw = output_shape(h, w, cfg.min_size, cfg.max_size)
    img = resize_pil(bgr, nh, nw).astype(np.float32).transpose(2, 0, 1)
    mean = np.asarray(PIXEL_MEAN, np.float32).reshape(3, 1, 1)
    std = np.asarray(PIXEL_STD, np.float32).reshape(3, 1, 1)
    x = (img - mean) / std
    hp, wp = -(-nh // 32) * 32, -(-nw // 32) * 32
    out = np.zeros((3, hp, wp), np.float32)
    out[:, :nh, :nw] = x
    return out, (nh, nw)


# --------------------------------------------------------------------------------------------- boxes
def cell_anchors(size: float, ratios: Sequence[float]) -> np.ndarray:
    """DefaultAnchorGenerator._generate_cell_anchors (python doubles, then float32)."""
    out = []
    area = size ** 2.0
    for r in ratios:
        w = math.sqrt(area / r)
        h = r * w
        out.append([-w / 2.0, -h / 2.0, w / 2.0, h / 2.0])
    return np.asarray(out, np.float32)


def grid_anchors(h: int, w: int, stride: int, size: float, ratios) -> torch.Tensor:
    """[h * w * A, 4] in (y, x, anchor) order: shifts (x * stride, y * stride) + cell anchors, float32."""
    sx = torch.arange(0, w * stride, stride, dtype=torch.float32)
    sy = torch.arange(0, h * stride, stride, dtype=torch.float32)
    yy, xx = torch.meshgrid(sy, sx, indexing="ij")
    shifts = torch.stack([xx.reshape(-1), yy.reshape(-1), xx.reshape(-1), yy.reshape(-1)], 1)
    base = torch.from_numpy(cell_anchors(size, ratios))
    return (shifts.view(-1, 1, 4) + base.view(1, -1, 4)).reshape(-1, 4)


def apply_deltas(deltas: torch.Tensor, boxes: torch.Tensor, weights) -> torch.Tensor:
    """Box2BoxTransform.apply_deltas (float32; each product and sum rounded on its own)."""
    deltas = deltas.float()
    widths = boxes[:, 2] - boxes[:, 0]
    heights = boxes[:, 3] - boxes[:, 1]
    ctr_x = boxes[:, 0] + 0.5 * widths
    ctr_y = boxes[:, 1] + 0.5 * heights
    wx, wy, ww, wh = weights
    dx = deltas[:, 0::4] / wx
    dy = deltas[:, 1::4] / wy
    dw = torch.clamp(deltas[:, 2::4] / ww, max=SCALE_CLAMP)
    dh = torch.clamp(deltas[:, 3::4] / wh, max=SCALE_CLAMP)
    pcx = dx * widths[:, None] + ctr_x[:, None]
    pcy = dy * heights[:, None] + ctr_y[:, None]
    pw = torch.exp(dw) * widths[:, None]
    ph = torch.exp(dh) * heights[:, None]
    out = torch.stack((pcx - 0.5 * pw, pcy - 0.5 * ph, pcx + 0.5 * pw, pcy + 0.5 * ph), dim=-1)
    return out.reshape(deltas.shape)


def clip_boxes(b: torch.Tensor, h: float, w: float) -> torch.Tensor:
    """Boxes.clip((h, w))."""
    return torch.stack((b[:, 0].clamp(min=0, max=w), b[:, 1].clamp(min=0, max=h),
                        b[:, 2].clamp(min=0, max=w), b[:, 3].clamp(min=0, max=h)), -1)


def nonempty(b: torch.Tensor, thr: float = 0.0) -> torch.Tensor:
    return ((b[:, 2] - b[:, 0]) > thr) & ((b[:, 3] - b[:, 1]) > thr)


def nms(boxes: torch.Tensor, scores: torch.Tensor, thr: float) -> torch.Tensor:
    """torchvision nms: stable descending sort, greedy suppression of later boxes with IoU > thr; kept indices in
    score order."""
    n = boxes.shape[0]
    if n == 0:
        return torch.zeros(0, dtype=torch.int64)
    order = torch.sort(scores, descending=True, stable=True)[1]
    b = boxes[order]
    x1, y1, x2, y2 = b[:, 0], b[:, 1], b[:, 2], b[:, 3]
    area = (x2 - x1) * (y2 - y1)
    left = torch.maximum(x1[:, None], x1[None, :])
    right = torch.minimum(x2[:, None], x2[None, :])
    top = torch.maximum(y1[:, None], y1[None, :])
    bottom = torch.minimum(y2[:, None], y2[None, :])
    inter = torch.clamp(right - left, min=0) * torch.clamp(bottom - top, min=0)
    iou = inter / ((area[:, None] + area[None, :]) - inter)
    sup = (iou > thr).numpy()
    removed = np.zeros(n, bool)
    keep = []
    for i in range(n):
        if removed[i]:
            continue
        keep.append(i)
        removed[i + 1:] |= sup[i, i + 1:]
    return order[torch.as_tensor(keep, dtype=torch.int64)]


def batched_nms(boxes: torch.Tensor, scores: torch.Tensor, idxs: torch.Tensor, thr: float) -> torch.Tensor:
    """torchvision _batched_nms_coordinate_trick (detectron2.layers.batched_nms on float boxes)."""
    if boxes.numel() == 0:
        return torch.zeros(0, dtype=torch.int64)
    mx = boxes.max()
    offsets = idxs.to(boxes.dtype) * (mx + torch.tensor(1, dtype=boxes.dtype))
    return nms(boxes + offsets[:, None], scores, thr)


def topk_stable(x: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """The k largest values, ties by the lower index (libvge's rule; torch.topk leaves it unspecified)."""
    v, i = torch.sort(x, descending=True, stable=True)
    return v[:k], i[:k]


# --------------------------------------------------------------------------------------------- ROIAlign
def roi_align(feat: torch.Tensor, rois: torch.Tensor, scale: float, pooled: int = 7) -> torch.Tensor:
    """torchvision roi_align (aligned=True, sampling_ratio 0) on one image: feat [C, H, W] float32, rois [R, 4] (image
    coordinates) -> [R, C, pooled, pooled].  Sample positions / weights in float32 as roi_align_kernel.cpp computes
    them; each bin = (sum over its samples of w1 v1 + w2 v2 + w3 v3 + w4 v4) / count."""
    C_, H, W = feat.shape
    out = torch.zeros((rois.shape[0], C_, pooled, pooled), dtype=torch.float32)
    fl = feat.reshape(C_, H * W)
    sc = f32(scale)
    for r in range(rois.shape[0]):
        x1, y1, x2, y2 = (f32(v) for v in rois[r].tolist())
        sw, sh = f32(x1 * sc) - f32(0.5), f32(y1 * sc) - f32(0.5)
        ew, eh = f32(x2 * sc) - f32(0.5), f32(y2 * sc) - f32(0.5)
        rw, rh = f32(ew - sw), f32(eh - sh)
        bw, bh = f32(rw / f32(pooled)), f32(rh / f32(pooled))
        gh = int(math.ceil(rh / f32(pooled)))
        gw = int(math.ceil(rw / f32(pooled)))
        count = f32(max(gh * gw, 1))
        # sample coordinates along each axis: start + p * bin + (i + .5) * bin / grid
        def coords(start, b, g):
            p = np.arange(pooled, dtype=np.float32)[:, None]
            i = np.arange(max(g, 0), dtype=np.float32)[None, :]
            return (f32(start) + p * b) + ((i + f32(0.5)) * b) / f32(g)
        ys, xs = coords(sh, bh, gh), coords(sw, bw, gw)          # [7, gh], [7, gw]

        def lin(c, n):
            valid = ~((c < -1.0) | (c > n))
            c = np.where(c <= 0, f32(0), c).astype(np.float32)
            lo = np.floor(c).astype(np.int64)   # c >= 0
            edge = lo >= n - 1
            lo = np.where(edge, n - 1, lo)
            hi = np.where(edge, n - 1, lo + 1)
            c = np.where(edge, lo.astype(np.float32), c).astype(np.float32)
            l_ = (c - lo.astype(np.float32)).astype(np.float32)
            return valid, lo, hi, l_, (f32(1) - l_).astype(np.float32)
        vy, ylo, yhi, ly, hy = lin(ys, H)
        vx, xlo, xhi, lx, hx = lin(xs, W)
        acc = torch.zeros((C_, pooled, pooled), dtype=torch.float32)
        for iy in range(max(gh, 0)):
            for ix in range(max(gw, 0)):
                v = (vy[:, iy][:, None] & vx[:, ix][None, :])                           # [7, 7]
                w1 = torch.from_numpy((hy[:, iy][:, None] * hx[:, ix][None, :]) * v)
                w2 = torch.from_numpy((hy[:, iy][:, None] * lx[:, ix][None, :]) * v)
                w3 = torch.from_numpy((ly[:, iy][:, None] * hx[:, ix][None, :]) * v)
                w4 = torch.from_numpy((ly[:, iy][:, None] * lx[:, ix][None, :]) * v)
                yl, yh_ = ylo[:, iy][:, None], yhi[:, iy][:, None]
                xl, xh_ = xlo[:, ix][None, :], xhi[:, ix][None, :]
                p1 = torch.from_numpy((yl * W + xl).reshape(-1))
                p2 = torch.from_numpy((yl * W + xh_).reshape(-1))
                p3 = torch.from_numpy((yh_ * W + xl).reshape(-1))
                p4 = torch.from_numpy((yh_ * W + xh_).reshape(-1))
                t = ((w1.reshape(1, -1) * fl[:, p1] + w2.reshape(1, -1) * fl[:, p2]) + w3.reshape(1, -1) * fl[:, p3]) \
                    + w4.reshape(1, -1) * fl[:, p4]
                acc = acc + t.reshape(C_, pooled, pooled)
        out[r] = acc / count
    return out


def assign_levels(boxes: torch.Tensor, min_level=2, max_level=5, canonical_size=224, canonical_level=4) -> torch.Tensor:
    """ROIPooler assign_boxes_to_levels -> level index 0..3 (P2..P5)."""
    area = (boxes[:, 2] - boxes[:, 0]) * (boxes[:, 3] - boxes[:, 1])
    sizes = torch.sqrt(area)
    lv = torch.floor(canonical_level + torch.log2(sizes / canonical_size + 1e-8))
    return torch.clamp(lv, min=min_level, max=max_level).to(torch.int64) - min_level


# --------------------------------------------------------------------------------------------- the network
class OracleFrcnn:
    def __init__(self, sd: Dict[str, np.ndarray], cfg, bf16: bool = True):
        self.p = {k: torch.as_tensor(np.asarray(v, np.float32)) for k, v in sd.items()}
        self.c = cfg
        self.bf16 = bf16
        self._w = {}

    def r(self, x):
        return x.to(torch.bfloat16).float() if self.bf16 else x

    # conv weights: the FrozenBN fold in float32 (scale = gamma / sqrt(var + eps), W * scale, beta - mean * scale)
    def folded(self, name):
        if name not in self._w:
            p = self.p
            w = p[name + ".weight"]
            if name + ".norm.weight" in p:
                g, b = p[name + ".norm.weight"].numpy(), p[name + ".norm.bias"].numpy()
                mu, var = p[name + ".norm.running_mean"].numpy(), p[name + ".norm.running_var"].numpy()
                s = (g / np.sqrt(var + f32(BN_EPS))).astype(np.float32)
                w = torch.from_numpy((w.numpy() * s.reshape(-1, 1, 1, 1)).astype(np.float32))
                bias = torch.from_numpy((b - mu * s).astype(np.float32))
            else:
                bias = p.get(name + ".bias", torch.zeros(w.shape[0]))
            self._w[name] = (self.r(w), bias)
        return self._w[name]

    def conv(self, x, name, stride=1, pad=None, groups=1, relu=False, res=None):
        w, b = self.folded(name)
        k = w.shape[-1]
        y = F.conv2d(x, w, b, stride=stride, padding=k // 2 if pad is None else pad, groups=groups)
        if res is not None:
            y = y + res
        if relu:
            y = torch.relu(y)
        return self.r(y)

    def backbone(self, x):
        c = self.c
        bb = "backbone.bottom_up."
        x = self.conv(self.r(x), bb + "stem.conv1", stride=2, pad=3, relu=True)
        x = F.max_pool2d(x, kernel_size=3, stride=2, padding=1)
        feats = []
        for si, nb in enumerate(STAGE_BLOCKS[c.depth]):
            for b in range(nb):
                p = f"{bb}res{si + 2}.{b}"
                stride = 2 if (b == 0 and si > 0) else 1
                sc = self.conv(x, p + ".shortcut", stride=stride) if b == 0 else x
                t = self.conv(x, p + ".conv1", relu=True)
                t = self.conv(t, p + ".conv2", stride=stride, groups=c.groups, relu=True)
                x = self.conv(t, p + ".conv3", relu=True, res=sc)
            feats.append(x)
        return feats

    def fpn(self, feats):
        outs = [None] * 4
        prev = self.conv(feats[3], "backbone.fpn_lateral5")
        outs[3] = self.conv(prev, "backbone.fpn_output5")
        for lv in (4, 3, 2):
            td = F.interpolate(prev, scale_factor=2.0, mode="nearest")
            prev = self.conv(feats[lv - 2], f"backbone.fpn_lateral{lv}", res=td)
            outs[lv - 2] = self.conv(prev, f"backbone.fpn_output{lv}")
        outs.append(F.max_pool2d(outs[3], kernel_size=1, stride=2, padding=0))
        return outs   # P2..P6

    def rpn_head(self, p):
        """-> (logits [N, H*W*A], deltas [N, H*W*A, 4]) in detectron2's (y, x, anchor) order."""
        t = self.conv(p, "proposal_generator.rpn_head.conv", relu=True)
        w_o, b_o = self.folded("proposal_generator.rpn_head.objectness_logits")
        w_d, b_d = self.folded("proposal_generator.rpn_head.anchor_deltas")
        lo = F.conv2d(t, w_o, b_o)
        de = F.conv2d(t, w_d, b_d)
        N, A, H, W = lo.shape
        return lo.permute(0, 2, 3, 1).reshape(N, -1), de.view(N, A, 4, H, W).permute(0, 3, 4, 1, 2).reshape(N, -1, 4)

    def proposals(self, logits: List[torch.Tensor], deltas: List[torch.Tensor], image_size, shapes):
        """find_top_rpn_proposals for ONE image: logits[l] [H*W*A], deltas[l] [H*W*A, 4] -> (boxes [P, 4], logits [P])."""
        c = self.c
        bx, sc, lv = [], [], []
        for l, (lo, de) in enumerate(zip(logits, deltas)):
            h, w = shapes[l]
            k = min(c.rpn_pre_topk, lo.shape[0])
            v, i = topk_stable(lo, k)
            anc = grid_anchors(h, w, 4 * 2 ** l, c.anchor_sizes[l], c.aspect_ratios)[i]
            bx.append(apply_deltas(de[i], anc, (1.0, 1.0, 1.0, 1.0)))
            sc.append(v)
            lv.append(torch.full((k,), l, dtype=torch.int64))
        boxes, scores, lvl = torch.cat(bx), torch.cat(sc), torch.cat(lv)
        boxes = clip_boxes(boxes, image_size[0], image_size[1])
        keep = nonempty(boxes)
        boxes, scores, lvl = boxes[keep], scores[keep], lvl[keep]
        keep = batched_nms(boxes, scores, lvl, c.rpn_nms)[:c.rpn_post_topk]
        return boxes[keep], scores[keep]

    def box_features(self, pfeats: List[torch.Tensor], boxes: torch.Tensor) -> torch.Tensor:
        """ROIPooler over P2..P5 of ONE image ([C, H, W] each) -> [R, C, 7, 7] (bf16-rounded as stored)."""
        lvl = assign_levels(boxes)
        out = torch.zeros((boxes.shape[0], pfeats[0].shape[0], self.c.pool, self.c.pool))
        for l in range(4):
            sel = torch.nonzero(lvl == l).view(-1)
            if sel.numel():
                out[sel] = roi_align(pfeats[l], boxes[sel], 1.0 / (4 * 2 ** l), self.c.pool)
        return self.r(out)

    def box_head(self, bf: torch.Tensor):
        """-> (cls logits [R, K + 1], deltas [R, 4K]) float32."""
        p = self.p
        x = bf.flatten(1)

        def lin(x, name, relu):
            w, b = self.r(p[name + ".weight"]), p[name + ".bias"]
            y = x @ w.t() + b
            return self.r(torch.relu(y)) if relu else y
        x = lin(x, "roi_heads.box_head.fc1", True)
        x = lin(x, "roi_heads.box_head.fc2", True)
        return lin(x, "roi_heads.box_predictor.cls_score", False), lin(x, "roi_heads.box_predictor.bbox_pred", False)

    def inference(self, cls_logits, deltas, proposals, image_size):
        """fast_rcnn_inference_single_image -> (boxes [n, 4], scores [n], classes [n]) in the resized image."""
        c = self.c
        mx = cls_logits.max(dim=1, keepdim=True).values
        e = torch.exp(cls_logits - mx)
        probs = e / e.sum(dim=1, keepdim=True)
        boxes = apply_deltas(deltas, proposals, (10.0, 10.0, 5.0, 5.0))
        scores = probs[:, :-1]
        K = scores.shape[1]
        boxes = clip_boxes(boxes.reshape(-1, 4), image_size[0], image_size[1]).view(-1, K, 4)
        mask = scores > c.score_thresh
        inds = mask.nonzero()
        boxes = boxes[mask]
        scores = scores[mask]
        keep = batched_nms(boxes, scores, inds[:, 1], c.nms_thresh)[:c.det_per_img]
        return boxes[keep], scores[keep], inds[keep, 1]

    @staticmethod
    def postprocess(boxes, scores, classes, image_size, out_h, out_w):
        """detector_postprocess: scale to the frame, clip, drop empty boxes."""
        sx, sy = f32(out_w / image_size[1]), f32(out_h / image_size[0])
        b = boxes.clone()
        b[:, 0::2] *= float(sx)
        b[:, 1::2] *= float(sy)
        b = clip_boxes(b, out_h, out_w)
        k = nonempty(b)
        return b[k], scores[k], classes[k]

    def detect(self, frames_rgb: np.ndarray, taps: bool = False):
        """frames uint8 [F, H, W, 3] RGB -> per frame {boxes [n, 4] frame pixels, scores [n], classes [n]} (+ the
        intermediate tensors with taps=True)."""
        F_, H, W = frames_rgb.shape[:3]
        xs, sizes = zip(*(preprocess(f, self.c) for f in frames_rgb))
        x = torch.from_numpy(np.stack(xs))
        feats = self.backbone(x)
        P = self.fpn(feats)
        heads = [self.rpn_head(p) for p in P]
        shapes = [tuple(p.shape[-2:]) for p in P]
        res = []
        for n in range(F_):
            pb, ps = self.proposals([h[0][n] for h in heads], [h[1][n] for h in heads], sizes[n], shapes)
            bf = self.box_features([p[n] for p in P[:4]], pb)
            cl, de = self.box_head(bf)
            b, s, k = self.inference(cl, de, pb, sizes[n])
            fb, fs, fk = self.postprocess(b, s, k, sizes[n], H, W)
            d = {"boxes": fb, "scores": fs, "classes": fk}
            if taps:
                d.update(proposals=pb, proposal_logits=ps, cls_logits=cl, deltas=de, box_features=bf,
                         image_size=sizes[n], pre_boxes=b, pre_scores=s, pre_classes=k)
            res.append(d)
        if taps:
            return res, {"image": x, "P": P, "heads": heads, "feats": feats}
        return res


def gate_persons(det: dict, thresh: float = 0.5) -> int:
    """mesh_generator.py:106-108: the number of (pred_classes == 0) & (scores > 0.5) boxes."""
    return int(((det["classes"] == 0) & (det["scores"] > thresh)).sum())
