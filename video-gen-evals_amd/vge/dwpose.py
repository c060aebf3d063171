"""Per-frame 2-D whole-body keypoints (DWPose) on the GPU: the host side of include/vge_dwpose.h.

Mirrors the reference's keypoint extractor boundary -- modifications/process_video.py:59-91 running
``DWposeDetector`` (modifications/dwpose_init.py:37-69) on every frame and keeping
``flatten_first_person_no_padding`` (process_video.py:23-57) rows in ``keypoints.npy`` -- as
``DwposeExtractor.keypoints(frames, boxes, n_persons)`` returning the [F, 120] rows the scoring path reads.

DWPose's Wholebody = YOLOX-L person detector + RTMPose-l whole-body (dw-ll_ucoco_384: CSPNeXt-P5 backbone,
RTMCCHead with a gated-attention unit and SimCC x/y classifiers over 2x sub-pixel bins), followed by the
COCO-WholeBody -> OpenPose-18 conversion (neck = mean of the shoulders) and dwpose_init.py's normalisation
(coordinates / frame size, score < 0.3 -> -1).  All arithmetic runs in libvge's HIP kernels (vge_cnn.hip,
vge_pose_head.hip); there is no CPU path.
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
class RtmposeConfig:
    in_h: int = 384                  # model input 288 (w) x 384 (h)
    in_w: int = 288
    stem_ch: int = 64                # CSPNeXt-P5, widen 1.0 / deepen 1.0 (RTMPose-l)
    stage_ch: Tuple[int, int, int, int] = (128, 256, 512, 1024)
    stage_blocks: Tuple[int, int, int, int] = (3, 6, 6, 3)
    keypoints: int = 133             # COCO-WholeBody
    gau_hidden: int = 256
    gau_s: int = 128
    gau_e: int = 512                 # hidden * expansion_factor 2
    final_k: int = 7
    split: int = 2                   # simcc_split_ratio 2.0 -> 576 x-bins, 768 y-bins


RTMPOSE_L = RtmposeConfig()


@dataclass(frozen=True)
class YoloxConfig:
    in_size: int = 640      # onnxdet.inference_detector input_shape (640, 640)
    width: int = 64         # YOLOX-L: wid_mul 1.0 -> base channels 64 (dark2..dark5: 128, 256, 512, 1024)
    depth: int = 3          # YOLOX-L: dep_mul 1.0 -> base depth 3 (CSP blocks 3, 9, 9, 3; PAFPN CSP 3)
    head_ch: int = 256      # int(256 * width)
    num_classes: int = 80   # COCO; only class 0 (person) can reach DWPose (class-aware NMS, cls_ind == 0 filter)


YOLOX_L = YoloxConfig()
NMS_THR, SCORE_THR_DET, PERSON_THR = 0.45, 0.1, 0.3   # onnxdet.inference_detector


def yolox_flops(cfg: YoloxConfig = YOLOX_L) -> float:
    """Algorithmic 2 x MACs of every convolution of the detector as libvge runs it (class-0 cls_pred only)."""
    S, w0, d, hc = cfg.in_size, cfg.width, cfg.depth, cfg.head_ch
    fl = 0.0

    def cv(hw, cin, cout, k):
        nonlocal fl
        fl += 2.0 * hw * cin * cout * k * k

    def csp(hw, cin, cout, n):
        hid = cout // 2
        cv(hw, cin, hid, 1); cv(hw, cin, hid, 1); cv(hw, 2 * hid, cout, 1)
        for _ in range(n):
            cv(hw, hid, hid, 1); cv(hw, hid, hid, 3)

    s2, s4, s8, s16, s32 = (S // 2) ** 2, (S // 4) ** 2, (S // 8) ** 2, (S // 16) ** 2, (S // 32) ** 2
    cv(s2, 12, w0, 3)
    cv(s4, w0, 2 * w0, 3); csp(s4, 2 * w0, 2 * w0, d)
    cv(s8, 2 * w0, 4 * w0, 3); csp(s8, 4 * w0, 4 * w0, 3 * d)
    cv(s16, 4 * w0, 8 * w0, 3); csp(s16, 8 * w0, 8 * w0, 3 * d)
    cv(s32, 8 * w0, 16 * w0, 3); cv(s32, 16 * w0, 8 * w0, 1); cv(s32, 32 * w0, 16 * w0, 1); csp(s32, 16 * w0, 16 * w0, d)
    c3, c4, c5 = 4 * w0, 8 * w0, 16 * w0
    cv(s32, c5, c4, 1); csp(s16, 2 * c4, c4, d); cv(s16, c4, c3, 1); csp(s8, 2 * c3, c3, d)
    cv(s16, c3, c3, 3)  # bu_conv2 (stride 2: output positions at /16)
    csp(s16, 2 * c3, c4, d); cv(s32, c4, c4, 3); csp(s32, 2 * c4, c5, d)
    for hw, cin in ((s8, c3), (s16, c4), (s32, c5)):
        cv(hw, cin, hc, 1)
        for _ in range(4):
            cv(hw, hc, hc, 3)
        cv(hw, hc, 1 + 4 + 1, 1)
    return fl

MEAN_BGR = (123.675, 116.28, 103.53)   # onnxpose.preprocess normalises the cv2 BGR frame with these, in order
STD_BGR = (58.395, 57.12, 57.375)
BBOX_PADDING = 1.25
SCORE_THR = 0.3                        # dwpose_init.py:53-58 (subset < 0.3 -> invisible -> -1)

# COCO-WholeBody index (after wholebody.py inserts the neck at 17) of each OpenPose-18 body point:
# openpose_idx [1,2,3,4,6,7,8,9,10,12,13,14,15,16,17] <- mmpose_idx [17,6,8,10,7,9,12,14,16,13,15,2,1,4,3]
OPENPOSE18_FROM_WB = (0, 17, 6, 8, 10, 5, 7, 9, 12, 14, 16, 11, 13, 15, 2, 1, 4, 3)
LEFT_HAND = tuple(range(91, 112))     # candidate[:, 92:113] (post-insert) = COCO-WholeBody 91..111
RIGHT_HAND = tuple(range(112, 133))   # candidate[:, 113:]


def rtmpose_flops(cfg: RtmposeConfig = RTMPOSE_L) -> float:
    """Algorithmic MAC x 2 of the dense convolutions / Linears of one pose instance (GEMM-shaped work only:
    depthwise, pooling, channel attention and the GAU's token mixing are counted separately)."""
    h, w = cfg.in_h // 2, cfg.in_w // 2
    s0 = cfg.stem_ch
    fl = 2.0 * h * w * (3 * 9 * (s0 // 2) + (s0 // 2) * 9 * (s0 // 2) + (s0 // 2) * 9 * s0)
    cin = s0
    for i, (c, n) in enumerate(zip(cfg.stage_ch, cfg.stage_blocks)):
        h, w = (h + 1) // 2, (w + 1) // 2
        hw = h * w
        fl += 2.0 * hw * cin * 9 * c
        if i == 3:
            fl += 2.0 * hw * (c * (c // 2) + 2 * c * c)
        mid = c // 2
        fl += 2.0 * hw * (2 * c * mid + 2 * mid * c + n * (mid * 9 * mid + mid * mid))
        cin = c
    hw = (cfg.in_h // 32) * (cfg.in_w // 32)
    fl += 2.0 * hw * cin * cfg.final_k ** 2 * cfg.keypoints
    K, H = cfg.keypoints, cfg.gau_hidden
    fl += 2.0 * K * (hw * H + H * (2 * cfg.gau_e + cfg.gau_s) + cfg.gau_e * H + H * cfg.split * (cfg.in_w + cfg.in_h))
    fl += 2.0 * K * K * (cfg.gau_s + cfg.gau_e)
    return fl


def box_center_scale(box, in_w: int, in_h: int) -> Tuple[np.ndarray, np.ndarray]:
    """onnxpose.bbox_xyxy2cs(padding=1.25) + _fix_aspect_ratio(w / h of the model input), float64 like numpy."""
    x0, y0, x1, y1 = (float(v) for v in box)
    center = np.array([x0 + x1, y0 + y1]) * 0.5
    w, h = (x1 - x0) * BBOX_PADDING, (y1 - y0) * BBOX_PADDING
    ar = in_w / in_h
    scale = np.array([w, w / ar]) if w > h * ar else np.array([h * ar, h])
    return center, scale


class RtmposeConfigC(C.Structure):
    _fields_ = [("in_h", C.c_int), ("in_w", C.c_int), ("stem_ch", C.c_int), ("stage_ch", C.c_int * 4),
                ("stage_blocks", C.c_int * 4), ("keypoints", C.c_int), ("gau_hidden", C.c_int), ("gau_s", C.c_int),
                ("gau_e", C.c_int), ("final_k", C.c_int), ("split", C.c_int)]


class YoloxConfigC(C.Structure):
    _fields_ = [(k, C.c_int) for k in ("in_size", "width", "depth", "head_ch", "num_classes")]


def _ycfg_c(cfg: YoloxConfig) -> YoloxConfigC:
    return YoloxConfigC(cfg.in_size, cfg.width, cfg.depth, cfg.head_ch, cfg.num_classes)


def _cfg_c(cfg: RtmposeConfig) -> RtmposeConfigC:
    return RtmposeConfigC(cfg.in_h, cfg.in_w, cfg.stem_ch, (C.c_int * 4)(*cfg.stage_ch),
                          (C.c_int * 4)(*cfg.stage_blocks), cfg.keypoints, cfg.gau_hidden, cfg.gau_s, cfg.gau_e,
                          cfg.final_k, cfg.split)


def _sig(lib):
    if getattr(lib, "_dwpose_sig", False):
        return lib
    vp, i32, i64 = C.c_void_p, C.c_int, C.c_long
    sig = {
        "vge_dwpose_create": [C.POINTER(RtmposeConfigC), C.POINTER(L.TensorView), i32, C.POINTER(vp)],
        "vge_dwpose_reserve": [vp, i32],
        "vge_dwpose_destroy": [vp],
        "vge_dwpose_keypoints": [vp, vp, i32, i32, i32, vp, i32, vp, vp, vp, vp, vp],
        "vge_dwpose_profile_begin": [vp, i32],
        "vge_dwpose_profile_read": [vp, C.POINTER(C.c_double), C.POINTER(C.c_int), C.POINTER(C.c_double)],
        "vge_op_conv_bf16": [vp, i64, vp, vp, vp, i64, vp, i64, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32,
                             i32, i32, vp],
        "vge_yolox_create": [C.POINTER(YoloxConfigC), C.POINTER(L.TensorView), i32, C.POINTER(vp)],
        "vge_yolox_reserve": [vp, i32],
        "vge_yolox_destroy": [vp],
        "vge_yolox_detect": [vp, vp, i32, i32, i32, vp, vp, vp, vp],
        "vge_yolox_detect_scored": [vp, vp, i32, i32, i32, vp, vp, vp, vp, vp],
        "vge_yolox_profile_begin": [vp, i32],
        "vge_yolox_profile_read": [vp, C.POINTER(C.c_double), C.POINTER(C.c_int), C.POINTER(C.c_double)],
    }
    for name, args in sig.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = C.c_int
    lib._dwpose_sig = True
    return lib


def _views(state_dict: Dict[str, np.ndarray]):
    keep, views = [], []
    for k, v in state_dict.items():
        a = np.ascontiguousarray(np.asarray(v, dtype=np.float32))
        keep.append(a)
        tv = L.TensorView()
        tv.name = k.encode()
        tv.data = a.ctypes.data
        tv.ndim = a.ndim
        for i, s in enumerate(a.shape[:4]):
            tv.shape[i] = s
        views.append(tv)
    return keep, (L.TensorView * len(views))(*views), len(views)


class DwposeExtractor:
    """One RTMPose whole-body model resident in HBM (BN-folded bf16 NHWC weights) + its activation workspace."""

    def __init__(self, state_dict: Dict[str, np.ndarray], cfg: RtmposeConfig = RTMPOSE_L, device="cuda",
                 max_instances: int = 64):
        self.lib = _sig(L.load())
        self.cfg = cfg
        self.device = torch.device(device)
        keep, arr, n = _views(state_dict)
        h = C.c_void_p()
        cc = _cfg_c(cfg)
        with torch.cuda.device(self.device):
            L.check(self.lib.vge_dwpose_create(C.byref(cc), arr, n, C.byref(h)), "vge_dwpose_create")
        del keep
        self.h = h
        self.max_instances = 0
        self.reserve(max_instances)

    def reserve(self, max_instances: int) -> None:
        if max_instances > self.max_instances:
            with torch.cuda.device(self.device):
                L.check(self.lib.vge_dwpose_reserve(self.h, int(max_instances)), "vge_dwpose_reserve")
            self.max_instances = max_instances

    @staticmethod
    def instances(n_persons: np.ndarray) -> int:
        n = np.asarray(n_persons)
        return int(np.where(n == 0, 1, np.minimum(n, 2)).sum())

    def keypoints(self, frames: torch.Tensor, boxes: Optional[np.ndarray] = None,
                  n_persons: Optional[np.ndarray] = None, out: Optional[torch.Tensor] = None,
                  simcc: Optional[torch.Tensor] = None, lv: Optional[torch.Tensor] = None) -> torch.Tensor:
        """frames: uint8 [F, H, W, 3] RGB on the device; boxes: host float [F, P, 4] xyxy pixels in detector order;
        n_persons: host int [F] (default 0 = whole frame).  Returns float32 [F, 120]: the keypoints.npy rows of
        process_video.py (body 18 x (x, y) of person 0, then two 21-point hands, coordinates / (W, H), -1 where
        the score is < 0.3)."""
        if frames.dtype != torch.uint8 or frames.dim() != 4 or frames.shape[3] != 3:
            raise L.VgeError("frames must be uint8 [F,H,W,3]")
        F_, H_, W_ = (int(v) for v in frames.shape[:3])
        npers = np.zeros(F_, np.int32) if n_persons is None else np.ascontiguousarray(n_persons, dtype=np.int32)
        if npers.shape != (F_,):
            raise L.VgeError("n_persons must be [F]")
        P = 0
        bx = None
        if boxes is not None:
            bx = np.ascontiguousarray(boxes, dtype=np.float32)
            if bx.ndim != 3 or bx.shape[0] != F_ or bx.shape[2] != 4:
                raise L.VgeError("boxes must be [F, P, 4]")
            P = int(bx.shape[1])
        self.reserve(max(self.instances(npers), 1))
        if out is None:
            out = torch.empty((F_, 120), device=frames.device, dtype=torch.float32)
        L.check(self.lib.vge_dwpose_keypoints(self.h, _ptr(frames), F_, H_, W_, bx.ctypes.data if bx is not None else None,
                                              P, npers.ctypes.data, _ptr(out), _ptr(simcc) if simcc is not None else None,
                                              _ptr(lv) if lv is not None else None, _stream(frames.device)),
                "vge_dwpose_keypoints")
        return out

    def profile_begin(self, max_calls: int) -> None:
        L.check(self.lib.vge_dwpose_profile_begin(self.h, int(max_calls)), "vge_dwpose_profile_begin")

    def profile_read(self):
        ms = (C.c_double * 3)()
        n = C.c_int()
        fl = C.c_double()
        L.check(self.lib.vge_dwpose_profile_read(self.h, ms, C.byref(n), C.byref(fl)), "vge_dwpose_profile_read")
        return {"gemm": ms[0], "dw_pool_attn_prep": ms[1], "head_misc": ms[2]}, n.value, fl.value

    def close(self) -> None:
        if self.h:
            self.lib.vge_dwpose_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class YoloxDetector:
    """DWPose's YOLOX person detector resident in HBM (onnxdet.inference_detector restated; person class only)."""

    def __init__(self, state_dict: Dict[str, np.ndarray], cfg: YoloxConfig = YOLOX_L, device="cuda", chunk: int = 32):
        self.lib = _sig(L.load())
        self.cfg = cfg
        self.device = torch.device(device)
        keep, arr, n = _views(state_dict)
        h = C.c_void_p()
        cc = _ycfg_c(cfg)
        with torch.cuda.device(self.device):
            L.check(self.lib.vge_yolox_create(C.byref(cc), arr, n, C.byref(h)), "vge_yolox_create")
            del keep
            self.h = h
            L.check(self.lib.vge_yolox_reserve(self.h, int(chunk)), "vge_yolox_reserve")

    @property
    def anchors(self) -> int:
        S = self.cfg.in_size
        return (S // 8) ** 2 + (S // 16) ** 2 + (S // 32) ** 2

    def detect(self, frames: torch.Tensor, cand: Optional[torch.Tensor] = None, with_scores: bool = False):
        """frames uint8 [F, H, W, 3] RGB on the device -> (boxes float [F, 2, 4] xyxy frame pixels of persons 0 and 1,
        n_persons int32 [F] = min(count, 2)), both on the device (inference_detector's final_boxes, first two);
        with_scores: + scores float [F, 2] of those persons (0 where absent; vge_yolox_detect_scored)."""
        if frames.dtype != torch.uint8 or frames.dim() != 4 or frames.shape[3] != 3:
            raise L.VgeError("frames must be uint8 [F,H,W,3]")
        F_, H_, W_ = (int(v) for v in frames.shape[:3])
        boxes = torch.empty((F_, 2, 4), device=frames.device, dtype=torch.float32)
        npers = torch.empty((F_,), device=frames.device, dtype=torch.int32)
        scores = torch.empty((F_, 2), device=frames.device, dtype=torch.float32) if with_scores else None
        L.check(self.lib.vge_yolox_detect_scored(self.h, _ptr(frames), F_, H_, W_, _ptr(boxes), _ptr(npers),
                                                 _ptr(scores) if with_scores else None,
                                                 _ptr(cand) if cand is not None else None, _stream(frames.device)),
                "vge_yolox_detect")
        return (boxes, npers, scores) if with_scores else (boxes, npers)

    def profile_begin(self, max_calls: int) -> None:
        L.check(self.lib.vge_yolox_profile_begin(self.h, int(max_calls)), "vge_yolox_profile_begin")

    def profile_read(self):
        ms = (C.c_double * 2)()
        n = C.c_int()
        fl = C.c_double()
        L.check(self.lib.vge_yolox_profile_read(self.h, ms, C.byref(n), C.byref(fl)), "vge_yolox_profile_read")
        return {"gemm": ms[0], "other": ms[1]}, n.value, fl.value

    def close(self) -> None:
        if self.h:
            self.lib.vge_yolox_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Wholebody:
    """DWposeDetector's per-frame path (dwpose_init.py:37-69 -> process_video.py:23-57): YOLOX persons -> RTMPose on
    persons 0 / 1 (whole frame when none) -> keypoints.npy rows [F, 120].  The person counts and boxes cross to the
    host once per call (the instance table of the pose model), as the reference's numpy NMS output does."""

    def __init__(self, det: YoloxDetector, pose: DwposeExtractor):
        self.det, self.pose = det, pose
        self._pin_b = self._pin_n = None

    def __call__(self, frames: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        boxes, npers = self.det.detect(frames)
        F_ = int(frames.shape[0])
        if self._pin_b is None or self._pin_b.shape[0] < F_:
            self._pin_b = torch.empty((F_, 2, 4), dtype=torch.float32, pin_memory=True)
            self._pin_n = torch.empty((F_,), dtype=torch.int32, pin_memory=True)
        hb, hn = self._pin_b[:F_], self._pin_n[:F_]
        hb.copy_(boxes, non_blocking=True)
        hn.copy_(npers, non_blocking=True)
        torch.cuda.current_stream(frames.device).synchronize()
        return self.pose.keypoints(frames, hb.numpy(), hn.numpy(), out=out)


# ---- op-level entry point (parity tests) ----------------------------------------------------------
def pack_conv_weight(w: torch.Tensor) -> torch.Tensor:
    """[Cout, Cin, KH, KW] -> the kernel's bf16 [Npad, Kp] layout (k = (kh * KW + kw) * Cin + ci)."""
    Cout, Cin, KH, KW = w.shape
    Kp = -(-KH * KW * Cin // 32) * 32
    Np = -(-Cout // 256) * 256
    p = torch.zeros((Np, Kp), dtype=torch.bfloat16, device=w.device)
    p[:Cout, :KH * KW * Cin] = w.permute(0, 2, 3, 1).reshape(Cout, -1).to(torch.bfloat16)
    return p


def conv_bf16(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, stride: int = 1, pad: int = 0, act: str = "silu",
              out_f32: bool = False, res: Optional[torch.Tensor] = None, rscale: Optional[torch.Tensor] = None,
              out: Optional[torch.Tensor] = None, res_pre: bool = False) -> torch.Tensor:
    """x: bf16 NHWC [n, H, W, Cin] (contiguous); w: f32/bf16 [Cout, Cin, KH, KW] -> NHWC [n, Ho, Wo, Cout].
    act: none / silu / sigmoid / relu; res: bf16 added after the activation (res_pre: before it) or f32 x rscale."""
    lib = _sig(L.load())
    n, H, W, Cin = x.shape
    Cout, _, KH, KW = w.shape
    Ho, Wo = (H + 2 * pad - KH) // stride + 1, (W + 2 * pad - KW) // stride + 1
    wp = pack_conv_weight(w)
    bp = torch.zeros(wp.shape[0], dtype=torch.float32, device=x.device)
    bp[:Cout] = bias
    if out is None:
        out = torch.empty((n, Ho, Wo, Cout), dtype=torch.float32 if out_f32 else torch.bfloat16, device=x.device)
    mode = 0 if res is None else ((3 if res_pre else 1) if res.dtype == torch.bfloat16 else 2)
    rs = None
    if mode == 2:
        rs = torch.zeros(wp.shape[0], dtype=torch.float32, device=x.device)
        rs[:Cout] = rscale
    actc = {"none": 0, "silu": 1, "sigmoid": 2, "relu": 3}[act]
    L.check(lib.vge_op_conv_bf16(_ptr(x), Cin, _ptr(wp), _ptr(bp), _ptr(out), Cout, _ptr(res) if res is not None else None,
                                 Cout if res is not None else 0, _ptr(rs) if rs is not None else None, n, H, W, Cin, KH, KW,
                                 stride, pad, Cout, actc, int(out_f32), mode, _stream(x.device)), "vge_op_conv_bf16")
    return out
