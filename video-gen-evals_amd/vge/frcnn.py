"""TokenHMR's single-person gate detector on the GPU: the host side of include/vge_frcnn.h.

The reference gates every frame of a video on detectron2's COCO Faster R-CNN X101-32x8d-FPN before running TokenHMR
(modifications/mesh_generator.py:69-73 build it, 103-117 apply it: a frame is used iff exactly one ``pred_classes ==
0`` instance has ``scores > 0.5``; its box is the crop box).  ``FrcnnDetector.detect(frames)`` is that predictor on a
batch of frames: the instances (boxes in frame pixels, scores, classes) and, per frame, the gate's person count and
the first person boxes.  All arithmetic runs in libvge's HIP kernels (vge_cnn.hip implicit-GEMM convolutions,
vge_frcnn_kernels.hip); there is no CPU path.  Parity vs detectron2's trained model is unpinned (weights and code
absent offline): tests/test_frcnn.py checks it against oracle/frcnn.py, the torch restatement of the same inference.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from . import lib as L
from .ops import _ptr, _stream


@dataclass(frozen=True)
class FrcnnConfig:
    """COCO-Detection/faster_rcnn_X_101_32x8d_FPN_3x.yaml on detectron2's defaults (mesh_generator.py:69-73)."""
    min_size: int = 800              # INPUT.MIN_SIZE_TEST
    max_size: int = 1333             # INPUT.MAX_SIZE_TEST
    depth: int = 101                 # RESNETS.DEPTH (blocks 3, 4, 23, 3)
    groups: int = 32                 # RESNETS.NUM_GROUPS
    width_per_group: int = 8         # RESNETS.WIDTH_PER_GROUP
    stem_ch: int = 64
    res2_ch: int = 256
    fpn_ch: int = 256
    anchor_sizes: Tuple[int, ...] = (32, 64, 128, 256, 512)
    aspect_ratios: Tuple[float, ...] = (0.5, 1.0, 2.0)
    rpn_pre_topk: int = 1000         # RPN.PRE_NMS_TOPK_TEST
    rpn_post_topk: int = 1000        # RPN.POST_NMS_TOPK_TEST
    rpn_nms: float = 0.7
    pool: int = 7                    # ROI_BOX_HEAD.POOLER_RESOLUTION
    fc_dim: int = 1024
    num_classes: int = 80
    score_thresh: float = 0.25       # mesh_generator.py:71
    nms_thresh: float = 0.5          # ROI_HEADS.NMS_THRESH_TEST
    det_per_img: int = 100           # TEST.DETECTIONS_PER_IMAGE
    gate_thresh: float = 0.5         # mesh_generator.py:106


FRCNN_X101 = FrcnnConfig()


class FrcnnConfigC(C.Structure):
    _fields_ = [("min_size", C.c_int), ("max_size", C.c_int), ("depth", C.c_int), ("groups", C.c_int),
                ("width_per_group", C.c_int), ("stem_ch", C.c_int), ("res2_ch", C.c_int), ("fpn_ch", C.c_int),
                ("rpn_pre_topk", C.c_int), ("rpn_post_topk", C.c_int), ("rpn_nms", C.c_float), ("fc_dim", C.c_int),
                ("num_classes", C.c_int), ("score_thresh", C.c_float), ("nms_thresh", C.c_float),
                ("det_per_img", C.c_int), ("gate_thresh", C.c_float)]


class FrcnnTapsC(C.Structure):
    _fields_ = [("resized", C.c_void_p), ("fpn", C.c_void_p * 5), ("rpn", C.c_void_p * 5), ("proposals", C.c_void_p),
                ("n_proposals", C.c_void_p), ("box_features", C.c_void_p), ("head", C.c_void_p),
                ("pre_dets", C.c_void_p), ("n_pre_dets", C.c_void_p)]


def _cfg_c(cfg: FrcnnConfig) -> FrcnnConfigC:
    return FrcnnConfigC(cfg.min_size, cfg.max_size, cfg.depth, cfg.groups, cfg.width_per_group, cfg.stem_ch,
                        cfg.res2_ch, cfg.fpn_ch, cfg.rpn_pre_topk, cfg.rpn_post_topk, cfg.rpn_nms, cfg.fc_dim,
                        cfg.num_classes, cfg.score_thresh, cfg.nms_thresh, cfg.det_per_img, cfg.gate_thresh)


def _sig(lib):
    if getattr(lib, "_frcnn_sig", False):
        return lib
    vp, i32 = C.c_void_p, C.c_int
    sig = {
        "vge_frcnn_create": [C.POINTER(FrcnnConfigC), C.POINTER(L.TensorView), i32, C.POINTER(vp)],
        "vge_frcnn_reserve": [vp, i32, i32, i32],
        "vge_frcnn_destroy": [vp],
        "vge_frcnn_shapes": [vp, i32, i32, C.POINTER(C.c_int)],
        "vge_frcnn_detect": [vp, vp, i32, i32, i32, vp, vp, vp, vp, C.POINTER(FrcnnTapsC), vp],
        "vge_frcnn_profile_begin": [vp, i32],
        "vge_frcnn_profile_read": [vp, C.POINTER(C.c_double), C.POINTER(C.c_int), C.POINTER(C.c_double)],
    }
    for k, a in sig.items():
        getattr(lib, k).argtypes = a
        getattr(lib, k).restype = C.c_int
    lib._frcnn_sig = True
    return lib


def _flops(cfg: FrcnnConfig, hp: int, wp: int) -> Tuple[float, float]:
    """Algorithmic 2 x MACs per frame padded to hp x wp: (backbone + FPN + RPN convolutions, box-head GEMMs over
    rpn_post_topk proposals); grouped 3x3 convolutions at their grouped size."""
    blocks = {50: (3, 4, 6, 3), 101: (3, 4, 23, 3), 152: (3, 8, 36, 3)}[cfg.depth]
    fl = 0.0

    def cv(px, cin, cout, k, g=1):
        nonlocal fl
        fl += 2.0 * px * (cin // g) * cout * k * k

    px = (hp // 2) * (wp // 2)
    cv(px, 3, cfg.stem_ch, 7)
    h, w = hp // 4, wp // 4
    cin, width, out = cfg.stem_ch, cfg.groups * cfg.width_per_group, cfg.res2_ch
    for s, nb in enumerate(blocks):
        for b in range(nb):
            st = 2 if (b == 0 and s > 0) else 1
            ho, wo = (h - 1) // st + 1, (w - 1) // st + 1
            if b == 0:
                cv(ho * wo, cin, out, 1)
            cv(h * w, cin if b == 0 else out, width, 1)
            cv(ho * wo, width, width, 3, cfg.groups)
            cv(ho * wo, width, out, 1)
            h, w = ho, wo
        cin, width, out = out, width * 2, out * 2
    F = cfg.fpn_ch
    lv = [(hp >> (l + 2)) * (wp >> (l + 2)) for l in range(4)]
    p6 = (((hp >> 5) - 1) // 2 + 1) * (((wp >> 5) - 1) // 2 + 1)
    for l in range(4):
        cv(lv[l], cfg.res2_ch << l, F, 1)
        cv(lv[l], F, F, 3)
    for px in lv + [p6]:
        cv(px, F, F, 3)
        cv(px, F, 15, 1)
    backbone = fl
    P = cfg.rpn_post_topk
    head = 2.0 * P * (F * 49 * cfg.fc_dim + cfg.fc_dim * cfg.fc_dim + cfg.fc_dim * (5 * cfg.num_classes + 1))
    return backbone, head


class FrcnnDetector:
    """detectron2 DefaultPredictor(faster_rcnn_X_101_32x8d_FPN_3x) resident in HBM: FrozenBN-folded bf16 NHWC
    weights + a chunk workspace.  chunk: frames per workspace pass (larger chunks fill the GPU better: 256 frames of
    256 x 256 take 260 / 252 / 244 ms at chunks of 32 / 32 / 64 on one box); capped where a layer's row count or an
    elementwise kernel's thread count would pass 2^31 (`max_chunk`: 838 frames at detectron2's 800-pixel size; every
    activation is addressed through 64-bit offsets)."""

    def __init__(self, state_dict: Dict[str, np.ndarray], cfg: FrcnnConfig = FRCNN_X101, device="cuda",
                 chunk: int = 64, frame_hw: Tuple[int, int] = (256, 256)):
        from .dwpose import _views
        self.lib = _sig(L.load())
        self.cfg = cfg
        self.device = torch.device(device)
        keep, arr, n = _views(state_dict)
        h = C.c_void_p()
        cc = _cfg_c(cfg)
        with torch.cuda.device(self.device):
            L.check(self.lib.vge_frcnn_create(C.byref(cc), arr, n, C.byref(h)), "vge_frcnn_create")
            del keep
            self.h = h
            self.chunk_req = int(chunk)
            self.chunk = min(self.chunk_req, self.max_chunk(*frame_hw))
            L.check(self.lib.vge_frcnn_reserve(self.h, self.chunk, int(frame_hw[0]), int(frame_hw[1])),
                    "vge_frcnn_reserve")
            self.frame_hw = (int(frame_hw[0]), int(frame_hw[1]))

    def max_chunk(self, H: int, W: int) -> int:
        """The largest chunk vge_frcnn_reserve accepts for H x W frames (rows per layer and threads per elementwise
        launch under 2^31, as vge_frcnn_reserve checks)."""
        sh = self.shapes(H, W)
        (hp, wp), (h4, w4) = sh["padded"], sh["levels"][0]
        c = self.cfg
        per = max(hp * wp, (hp // 2) * (wp // 2) * c.stem_ch // 8,
                  h4 * w4 * max(c.res2_ch, 2 * c.groups * c.width_per_group, c.fpn_ch) // 8)
        return max(1, ((1 << 31) - 1) // per)

    def shapes(self, H: int, W: int) -> Dict[str, object]:
        out = (C.c_int * 15)()
        L.check(self.lib.vge_frcnn_shapes(self.h, int(H), int(W), out), "vge_frcnn_shapes")
        return {"resized": (out[0], out[1]), "padded": (out[2], out[3]),
                "levels": [(out[4 + 2 * l], out[5 + 2 * l]) for l in range(5)], "ld_head": out[14]}

    def flops(self, H: int, W: int) -> Tuple[float, float]:
        hp, wp = self.shapes(H, W)["padded"]
        return _flops(self.cfg, hp, wp)

    def make_taps(self, F: int, H: int, W: int) -> Dict[str, torch.Tensor]:
        """Device tensors for every parity tap of `F` frames of H x W."""
        sh = self.shapes(H, W)
        dev, P, c = self.device, self.cfg.rpn_post_topk, self.cfg
        nh, nw = sh["resized"]
        t = {"resized": torch.empty((F, nh, nw, 3), dtype=torch.uint8, device=dev),
             "fpn": [torch.empty((F, h, w, c.fpn_ch), dtype=torch.bfloat16, device=dev) for h, w in sh["levels"]],
             "rpn": [torch.empty((F, h, w, 16), dtype=torch.float32, device=dev) for h, w in sh["levels"]],
             "proposals": torch.zeros((F, P, 5), dtype=torch.float32, device=dev),
             "n_proposals": torch.zeros((F,), dtype=torch.int32, device=dev),
             "box_features": torch.empty((F, P, 49, c.fpn_ch), dtype=torch.bfloat16, device=dev),
             "head": torch.empty((F, P, sh["ld_head"]), dtype=torch.float32, device=dev),
             "pre_dets": torch.zeros((F, c.det_per_img, 6), dtype=torch.float32, device=dev),
             "n_pre_dets": torch.zeros((F,), dtype=torch.int32, device=dev)}
        return t

    @staticmethod
    def _taps_c(t: Dict[str, torch.Tensor]) -> FrcnnTapsC:
        tc = FrcnnTapsC()
        for k in ("resized", "proposals", "n_proposals", "box_features", "head", "pre_dets", "n_pre_dets"):
            if k in t:
                setattr(tc, k, _ptr(t[k]))
        for k in ("fpn", "rpn"):
            for l, x in enumerate(t.get(k, [])):
                getattr(tc, k)[l] = _ptr(x)
        return tc

    def detect(self, frames: torch.Tensor, taps: Optional[Dict[str, torch.Tensor]] = None):
        """frames uint8 [F, H, W, 3] RGB on the device -> dict of device tensors:
        dets [F, det_per_img, 6] (x1 y1 x2 y2 frame pixels, score, class; the first n_dets[f] rows are the predictor's
        instances in score order), n_dets [F], person [F, 2, 5] (first two class-0 instances: box, score),
        n_person [F] (class-0 instances with score > 0.5: the gate keeps a frame iff it is 1)."""
        if frames.dtype != torch.uint8 or frames.dim() != 4 or frames.shape[3] != 3 or not frames.is_contiguous():
            raise L.VgeError("frames must be contiguous uint8 [F,H,W,3]")
        F_, H_, W_ = (int(v) for v in frames.shape[:3])
        if (H_, W_) != self.frame_hw:  # a new frame size: the workspace is rebuilt at a chunk that fits it
            self.chunk = min(self.chunk_req, self.max_chunk(H_, W_))
            with torch.cuda.device(self.device):
                L.check(self.lib.vge_frcnn_reserve(self.h, self.chunk, H_, W_), "vge_frcnn_reserve")
            self.frame_hw = (H_, W_)
        dev = frames.device
        out = {"dets": torch.zeros((F_, self.cfg.det_per_img, 6), dtype=torch.float32, device=dev),
               "n_dets": torch.empty((F_,), dtype=torch.int32, device=dev),
               "person": torch.empty((F_, 2, 5), dtype=torch.float32, device=dev),
               "n_person": torch.empty((F_,), dtype=torch.int32, device=dev)}
        tc = self._taps_c(taps) if taps is not None else None
        L.check(self.lib.vge_frcnn_detect(self.h, _ptr(frames), F_, H_, W_, _ptr(out["dets"]), _ptr(out["n_dets"]),
                                          _ptr(out["person"]), _ptr(out["n_person"]),
                                          C.byref(tc) if tc is not None else None, _stream(dev)),
                "vge_frcnn_detect")
        return out

    def profile_begin(self, max_calls: int) -> None:
        L.check(self.lib.vge_frcnn_profile_begin(self.h, int(max_calls)), "vge_frcnn_profile_begin")

    def profile_read(self):
        ms = (C.c_double * 3)()
        n = C.c_int()
        fl = (C.c_double * 2)()
        L.check(self.lib.vge_frcnn_profile_read(self.h, ms, C.byref(n), fl), "vge_frcnn_profile_read")
        return {"backbone_gemm": ms[0], "head_gemm": ms[1], "other": ms[2]}, n.value, (fl[0], fl[1])

    def close(self) -> None:
        if getattr(self, "h", None):
            self.lib.vge_frcnn_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
