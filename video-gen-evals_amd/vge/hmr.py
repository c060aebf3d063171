"""Per-frame mesh extraction (TokenHMR) on the GPU: the host side of include/vge_hmr.h.

Mirrors the reference's extractor boundary -- MeshGenerator.process_video (modifications/mesh_generator.py:
119-171) feeding SMPLTokenDecoderHead (modifications/token_head.py:180-246) and extract_mesh.py:35-43's npz
arrays -- as ``HmrExtractor.process_video(frames)`` returning {pose, global_orient, betas, vit} per frame, and
``extract_into`` writing straight into an HBM frame store for the scoring path (no npz round trip).
The detector gate (mesh_generator.py:103-117) and the crop warp are upstream of this boundary: frames arrive
as 256x256 RGB person crops.  All arithmetic runs in libvge's HIP kernels (vge_vit.hip); there is no CPU path.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import asdict, dataclass
from typing import Dict, Optional

import numpy as np
import torch

from . import lib as L
from .ops import _ptr, _stream


@dataclass(frozen=True)
class HmrConfig:
    in_h: int = 256
    in_w: int = 256
    img_h: int = 256
    img_w: int = 192
    patch: int = 16
    pad: int = 2
    embed_dim: int = 1280
    depth: int = 32
    heads: int = 16
    mlp_dim: int = 5120
    dec_dim: int = 1024
    dec_depth: int = 6
    dec_heads: int = 8
    dec_dim_head: int = 64
    dec_mlp: int = 1024
    tok_num: int = 160
    tok_classes: int = 2048
    tok_code_dim: int = 256


TOKENHMR = HmrConfig()  # ViT-H/16 backbone + 6-layer decoder (HMR2 / TokenHMR shapes)


class HmrConfigC(C.Structure):
    _fields_ = [(k, C.c_int) for k in HmrConfig.__dataclass_fields__]


def _cfg_c(cfg: HmrConfig) -> HmrConfigC:
    return HmrConfigC(**asdict(cfg))


def _sig(lib):
    if getattr(lib, "_hmr_sig", False):
        return lib
    vp, i32 = C.c_void_p, C.c_int
    sig = {
        "vge_hmr_create": [C.POINTER(HmrConfigC), C.POINTER(L.TensorView), i32, C.POINTER(vp)],
        "vge_hmr_reserve": [vp, i32],
        "vge_hmr_destroy": [vp],
        "vge_hmr_extract": [vp, vp, i32, vp, vp, vp, vp, vp],
        "vge_hmr_profile_begin": [vp, i32],
        "vge_hmr_profile_read": [vp, C.POINTER(C.c_double), C.POINTER(C.c_int), C.POINTER(C.c_double)],
        "vge_op_gemm_bf16": [i32, vp, C.c_long, vp, C.c_long, vp, C.c_long, vp, vp, C.c_long, vp, i32, i32, i32, i32,
                             vp],
        "vge_op_gemm_lib": [i32, vp, C.c_long, vp, C.c_long, vp, C.c_long, vp, vp, C.c_long, i32, i32, i32, vp],
        "vge_op_vit_attention": [vp, vp, i32, i32, i32, vp],
        "vge_hmr_crop": [vp, i32, i32, i32, vp, vp, i32, vp, vp],
        "vge_op_layernorm_bf16": [vp, vp, vp, vp, i32, i32, C.c_float, vp],
    }
    for name, args in sig.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = C.c_int
    lib._hmr_sig = True
    return lib


class HmrExtractor:
    """One TokenHMR model resident in HBM (bf16 weights) + its activation workspace."""

    def __init__(self, state_dict: Dict[str, np.ndarray], cfg: HmrConfig = TOKENHMR, device="cuda", max_frames: int = 256):
        self.lib = _sig(L.load())
        self.cfg = cfg
        self.device = torch.device(device)
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
        arr = (L.TensorView * len(views))(*views)
        h = C.c_void_p()
        cc = _cfg_c(cfg)
        with torch.cuda.device(self.device):
            L.check(self.lib.vge_hmr_create(C.byref(cc), arr, len(views), C.byref(h)), "vge_hmr_create")
        self.h = h
        self.max_frames = 0
        self.reserve(max_frames)

    def reserve(self, max_frames: int) -> None:
        if max_frames > self.max_frames:
            with torch.cuda.device(self.device):
                L.check(self.lib.vge_hmr_reserve(self.h, int(max_frames)), "vge_hmr_reserve")
            self.max_frames = max_frames

    def extract(self, frames: torch.Tensor, out: Optional[Dict[str, torch.Tensor]] = None) -> Dict[str, torch.Tensor]:
        """frames: uint8 [F, 256, 256, 3] RGB on the device -> {pose [F,207], global_orient [F,9], betas [F,10],
        vit [F, dec_dim]} float32 (the npz arrays of extract_mesh.py:35-43, flattened rotation matrices)."""
        if frames.dtype != torch.uint8 or frames.dim() != 4 or tuple(frames.shape[1:]) != (self.cfg.in_h, self.cfg.in_w, 3):
            raise L.VgeError(f"frames must be uint8 [F,{self.cfg.in_h},{self.cfg.in_w},3]")
        n = int(frames.shape[0])
        self.reserve(n)
        if out is None:
            dev = frames.device
            out = {"pose": torch.empty((n, 207), device=dev), "global_orient": torch.empty((n, 9), device=dev),
                   "betas": torch.empty((n, 10), device=dev), "vit": torch.empty((n, self.cfg.dec_dim), device=dev)}
        L.check(self.lib.vge_hmr_extract(self.h, _ptr(frames), n, _ptr(out["pose"]), _ptr(out["global_orient"]),
                                         _ptr(out["betas"]), _ptr(out["vit"]), _stream(frames.device)),
                "vge_hmr_extract")
        return out

    def process_video(self, frames: torch.Tensor) -> Dict[int, Dict[str, np.ndarray]]:
        """MeshGenerator.process_video's output shape (mesh_generator.py:160-169): {frame_idx: {pose [23,3,3],
        betas [10], global_orient [1,3,3], vit [1024]}} for frames that passed the (upstream) detector gate."""
        o = self.extract(frames)
        h = {k: v.cpu().numpy() for k, v in o.items()}
        return {i: {"pose": h["pose"][i].reshape(23, 3, 3), "betas": h["betas"][i],
                    "global_orient": h["global_orient"][i].reshape(1, 3, 3), "vit": h["vit"][i]}
                for i in range(frames.shape[0])}

    def profile_begin(self, max_calls: int) -> None:
        L.check(self.lib.vge_hmr_profile_begin(self.h, int(max_calls)), "vge_hmr_profile_begin")

    def profile_read(self):
        ms = (C.c_double * 4)()
        n = C.c_int()
        fl = C.c_double()
        L.check(self.lib.vge_hmr_profile_read(self.h, ms, C.byref(n), C.byref(fl)), "vge_hmr_profile_read")
        return {"gemm": ms[0], "attention": ms[1], "layernorm_patchify": ms[2], "head": ms[3]}, n.value, fl.value

    def close(self) -> None:
        if self.h:
            self.lib.vge_hmr_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---- op-level entry points (parity tests) ---------------------------------------------------------
EPI = {"bf16": 0, "gelu_bf16": 1, "res_f32": 2, "pe_f32": 3, "f32": 4}


def gemm_bf16(A: torch.Tensor, W: torch.Tensor, epi: str = "bf16", bias=None, res=None, pos=None, tokens: int = 192,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out = epilogue(A @ W^T) with A [M,K], W [N,K] bf16 device tensors (the extractor's GEMM kernel)."""
    lib = _sig(L.load())
    M, K = A.shape
    N = W.shape[0]
    if out is None:
        dt = torch.bfloat16 if epi in ("bf16", "gelu_bf16") else torch.float32
        out = torch.empty((M, N), device=A.device, dtype=dt)
    L.check(lib.vge_op_gemm_bf16(EPI[epi], _ptr(A), A.stride(0), _ptr(W), W.stride(0), _ptr(out), out.stride(0),
                                 _ptr(bias), _ptr(res), res.stride(0) if res is not None else 0, _ptr(pos), tokens,
                                 M, N, K, _stream(A.device)), "vge_op_gemm_bf16")
    return out


def gemm_lib(A: torch.Tensor, W: torch.Tensor, epi: str = "bf16", bias=None, res=None,
             out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The same product through the library path (hipBLASLt; vge_blaslt.cpp) for the "bf16", "res_f32" and "f32"
    epilogues; raises VGE_ERR_UNSUPPORTED for the others."""
    lib = _sig(L.load())
    M, K = A.shape
    N = W.shape[0]
    if out is None:
        out = torch.empty((M, N), device=A.device, dtype=torch.bfloat16 if epi == "bf16" else torch.float32)
    L.check(lib.vge_op_gemm_lib(EPI[epi], _ptr(A), A.stride(0), _ptr(W), W.stride(0), _ptr(out), out.stride(0),
                                _ptr(bias), _ptr(res), res.stride(0) if res is not None else 0, M, N, K,
                                _stream(A.device)), "vge_op_gemm_lib")
    return out


def vit_attention(qkv: torch.Tensor, heads: int) -> torch.Tensor:
    lib = _sig(L.load())
    rows, D3 = qkv.shape
    D = D3 // 3
    out = torch.empty((rows, D), device=qkv.device, dtype=torch.bfloat16)
    L.check(lib.vge_op_vit_attention(_ptr(qkv), _ptr(out), rows // 192, D, heads, _stream(qkv.device)),
            "vge_op_vit_attention")
    return out


def layernorm_bf16(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float) -> torch.Tensor:
    lib = _sig(L.load())
    rows, D = x.shape
    out = torch.empty((rows, D), device=x.device, dtype=torch.bfloat16)
    L.check(lib.vge_op_layernorm_bf16(_ptr(x), _ptr(out), _ptr(w), _ptr(b), rows, D, eps, _stream(x.device)),
            "vge_op_layernorm_bf16")
    return out


def crop_persons(frames: torch.Tensor, boxes, frame_of=None) -> torch.Tensor:
    """ViTDetDataset's person crop (mesh_generator.py:119-145; vge_hmr_crop): frames uint8 [F, H, W, 3] RGB on the
    device, boxes host float [n, 4] xyxy, frame_of host int [n] (None: crop i from frame i) -> uint8 [n, 256, 256, 3]
    device crops, the input of HmrExtractor.extract."""
    lib = _sig(L.load())
    if frames.dtype != torch.uint8 or frames.dim() != 4 or frames.shape[3] != 3:
        raise L.VgeError("frames must be uint8 [F,H,W,3]")
    b = np.ascontiguousarray(np.asarray(boxes, np.float32).reshape(-1, 4))
    n = b.shape[0]
    fo = None if frame_of is None else np.ascontiguousarray(np.asarray(frame_of, np.int32).reshape(-1))
    if fo is not None and fo.shape[0] != n:
        raise L.VgeError("frame_of must have one entry per box")
    out = torch.empty((n, 256, 256, 3), dtype=torch.uint8, device=frames.device)
    F_, H_, W_ = (int(v) for v in frames.shape[:3])
    L.check(lib.vge_hmr_crop(_ptr(frames), F_, H_, W_, b.ctypes.data, None if fo is None else fo.ctypes.data, n,
                             _ptr(out), _stream(frames.device)), "vge_hmr_crop")
    return out

