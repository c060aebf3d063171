"""ORACLE (test infrastructure only): torch CPU restatement of the TokenHMR per-frame extractor.

The reference runs TokenHMR through modifications/mesh_generator.py:119-171 (model(batch) on 256x256 person
crops, keeping pred_smpl_params body_pose / global_orient / betas / token_out) with the head of
modifications/token_head.py:180-246.  The backbone (HMR2 ViT-H/16), the cross-attention decoder
(HMR2 pose_transformer.TransformerDecoder) and the token classifier are third-party modules that are NOT in
/root/reference (TokenHMR / 4D-Humans at HEAD, no pinned version, no weights offline), so this file restates
their published structure:

  ViT (hmr2/models/backbones/vit.py)   x[:, :, :, 32:-32] crop, PatchEmbed Conv2d(3, E, 16, stride 16, pad 2),
                                       + pos_embed[:, 1:] + pos_embed[:, :1], blocks x = x + attn(norm1(x));
                                       x = x + mlp(norm2(x)) (LayerNorm eps 1e-6, qkv bias, exact GELU),
                                       last_norm
  TransformerDecoder (pose_transformer) to_token_embedding(zero token) + pos_embedding; layers of PreNorm
                                       self-attention (one token: softmax over one key = 1), PreNorm
                                       cross-attention to the 192 context tokens (dim_head 64, no q/kv bias),
                                       PreNorm FeedForward (Linear, GELU, Linear), LayerNorm eps 1e-5
  readouts (token_head.py:207-222)     decpose_grot / decpose_hands / decshape / deccam + the mean params
  TokenClassfier                       STAND-IN (its tokenizer is not in the reference): logits ->
                                       per-token softmax -> codebook -> linear decoder -> 21 x 6D body pose
  rot6d_to_rotmat (hmr2/utils/geometry) Gram-Schmidt with F.normalize (eps 1e-12)

Parity vs the upstream TokenHMR weights is UNPINNED (nothing in the reference fixes these numbers).  With
``bf16=True`` the restatement rounds to bfloat16 exactly where libvge's kernels store bf16 (GEMM operands,
LayerNorm outputs, attention probabilities), so the GPU path is compared against the same arithmetic up to
f32 summation order; with ``bf16=False`` it is the plain fp32 model (the bf16 deviation is reported).
"""
from __future__ import annotations

import math
from typing import Dict

import numpy as np
import torch
import torch.nn.functional as F

IMG_MEAN = (123.675, 116.28, 103.53)   # 255 * ImageNet mean (hmr2 DEFAULT_MEAN)
IMG_STD = (58.395, 57.12, 57.375)      # 255 * ImageNet std


def rot6d_to_rotmat(x: torch.Tensor) -> torch.Tensor:
    """hmr2.utils.geometry.rot6d_to_rotmat: [N, 6] -> [N, 3, 3]."""
    x = x.reshape(-1, 2, 3).permute(0, 2, 1).contiguous()
    a1, a2 = x[:, :, 0], x[:, :, 1]
    b1 = F.normalize(a1)
    b2 = F.normalize(a2 - torch.einsum("bi,bi->b", b1, a2).unsqueeze(-1) * b1)
    b3 = torch.cross(b1, b2, dim=-1)
    return torch.stack((b1, b2, b3), dim=-1)


class OracleHmr:
    def __init__(self, sd: Dict[str, np.ndarray], cfg, bf16: bool = True):
        self.p = {k: torch.as_tensor(np.asarray(v, np.float32)) for k, v in sd.items()}
        self.c = cfg
        self.bf16 = bf16

    def r(self, x: torch.Tensor) -> torch.Tensor:  # a bf16 storage point of the GPU path
        return x.to(torch.bfloat16).float() if self.bf16 else x

    def lin(self, x: torch.Tensor, key: str, bias: bool = True, w: torch.Tensor = None) -> torch.Tensor:
        W = self.p[key + ".weight"] if w is None else w
        y = self.r(x) @ self.r(W).t()
        if bias:
            y = y + self.p[key + ".bias"]
        return y

    def ln(self, x, key, eps):
        return self.r(F.layer_norm(x, (x.shape[-1],), self.p[key + ".weight"], self.p[key + ".bias"], eps=eps))

    def backbone(self, frames_u8: np.ndarray) -> torch.Tensor:
        """frames [F, 256, 256, 3] uint8 RGB -> context tokens [F, 192, E] (after last_norm)."""
        c, p = self.c, self.p
        img = torch.as_tensor(frames_u8).float().permute(0, 3, 1, 2)          # [F, 3, H, W]
        x0 = (c.in_w - c.img_w) // 2
        img = img[:, :, :, x0:x0 + c.img_w]
        mean = torch.tensor(IMG_MEAN).view(1, 3, 1, 1)
        std = torch.tensor(IMG_STD).view(1, 3, 1, 1)
        img = (img - mean) / std
        cols = F.unfold(img, kernel_size=c.patch, stride=c.patch, padding=c.pad)  # [F, 3*P*P, 192]
        cols = self.r(cols.transpose(1, 2))
        E = c.embed_dim
        Wpe = p["backbone.patch_embed.proj.weight"].reshape(E, -1)
        x = self.lin(cols, "backbone.patch_embed.proj", w=Wpe)
        pos = p["backbone.pos_embed"][0]
        x = x + pos[1:] + pos[:1]
        hd = E // c.heads
        Fn, T, _ = x.shape
        for i in range(c.depth):
            b = f"backbone.blocks.{i}."
            h = self.ln(x, b + "norm1", 1e-6)
            qkv = self.r(self.lin(h, b + "attn.qkv")).view(Fn, T, 3, c.heads, hd).permute(2, 0, 3, 1, 4)
            q, k, v = qkv[0], qkv[1], qkv[2]
            s = (q @ k.transpose(-2, -1)) / math.sqrt(hd)
            m = s.amax(-1, keepdim=True)
            e = torch.exp(s - m)
            den = e.sum(-1, keepdim=True)
            o = (self.r(e) @ v) / den
            o = self.r(o.transpose(1, 2).reshape(Fn, T, E))
            x = x + self.lin(o, b + "attn.proj")
            h = self.ln(x, b + "norm2", 1e-6)
            h = self.r(F.gelu(self.lin(h, b + "mlp.fc1")))
            x = x + self.lin(h, b + "mlp.fc2")
        return self.ln(x, "backbone.last_norm", 1e-6)

    def head(self, ctx: torch.Tensor):
        c, p = self.c, self.p
        Fn = ctx.shape[0]
        inner = c.dec_heads * 64
        t = "smpl_head.transformer."
        x = (p[t + "to_token_embedding.bias"] + p[t + "pos_embedding"][0, 0]).expand(Fn, -1).clone()
        for l in range(c.dec_depth):
            L = f"{t}transformer.layers.{l}."
            h = self.ln(x, L + "0.norm", 1e-5)
            wv = p[L + "0.fn.to_qkv.weight"][2 * inner:3 * inner]
            v = self.r(self.lin(h, L + "0.fn.to_qkv", bias=False, w=wv))
            x = x + self.lin(v, L + "0.fn.to_out.0")
            h = self.ln(x, L + "1.norm", 1e-5)
            q = self.r(self.lin(h, L + "1.fn.to_q", bias=False)).view(Fn, c.dec_heads, 1, 64)
            kv = self.r(self.lin(ctx, L + "1.fn.to_kv", bias=False))
            k = kv[..., :inner].reshape(Fn, -1, c.dec_heads, 64).transpose(1, 2)
            vv = kv[..., inner:].reshape(Fn, -1, c.dec_heads, 64).transpose(1, 2)
            a = ((q @ k.transpose(-2, -1)) * 0.125).softmax(-1)
            o = self.r((a @ vv).transpose(1, 2).reshape(Fn, inner))
            x = x + self.lin(o, L + "1.fn.to_out.0")
            h = self.ln(x, L + "2.norm", 1e-5)
            h = self.r(F.gelu(self.lin(h, L + "2.fn.net.0")))
            x = x + self.lin(h, L + "2.fn.net.3")
        token_out = x
        s = "smpl_head."
        grot = self.lin(x, s + "decpose_grot")
        hands = self.lin(x, s + "decpose_hands")
        shape = self.lin(x, s + "decshape")
        logits = self.lin(x, s + "decpose.cls").view(Fn * c.tok_num, c.tok_classes)
        probs = self.r(logits.softmax(-1))
        qz = self.r(probs @ self.r(p[s + "decpose.codebook"])).view(Fn, c.tok_num * c.tok_code_dim)
        bpose = self.lin(qz, s + "decpose.dec")
        body = torch.cat([grot, bpose, hands], -1) + p[s + "init_body_pose"]
        R = rot6d_to_rotmat(body).view(Fn, 24, 3, 3)
        betas = shape + p[s + "init_betas"]
        return {"global_orient": R[:, :1].reshape(Fn, 9), "pose": R[:, 1:].reshape(Fn, 207), "betas": betas,
                "vit": token_out}

    @torch.no_grad()
    def forward(self, frames_u8: np.ndarray):
        return self.head(self.backbone(frames_u8))


# ------------------------------------------------------------------------- the TokenHMR front end (crop + gate)
# ViTDetDataset (4D-Humans hmr2/datasets/vitdet_dataset.py, no pinned version; driven by
# modifications/mesh_generator.py:119-145) restated: rescale_factor 2.5, BBOX_SHAPE [192, 256], IMAGE_SIZE 256,
# skimage.filters.gaussian anti-aliasing (mode 'nearest', truncate 4) when the patch is downsampled > 2.2x,
# generate_image_patch_cv2 -> cv2.warpAffine(INTER_LINEAR, BORDER_CONSTANT 0).  cv2's bilinear is restated in
# float32 without contraction (the kernel vge_hmr_front.hip runs the same operations), rounded like a uint8 warp.

def expand_to_aspect_ratio(wh, target=(192, 256)):
    w, h = float(wh[0]), float(wh[1])
    wt, ht = target
    if h / w < ht / wt:
        return np.array([w, max(w * ht / wt, h)])
    return np.array([max(h * wt / ht, w), h])


def vitdet_geometry(box):
    """box xyxy -> (cx, cy, k = bbox_size / 256, sigma or 0) in ViTDetDataset's float32 / float64 arithmetic."""
    b = np.asarray(box, np.float32)
    c = (b[2:4] + b[0:2]) / np.float32(2.0)
    scale = np.float32(2.5) * (b[2:4] - b[0:2]) / np.float32(200.0)
    bbox = float(expand_to_aspect_ratio((float(scale[0] * np.float32(200)), float(scale[1] * np.float32(200)))).max())
    df = bbox / 256.0 / 2.0
    return float(c[0]), float(c[1]), np.float32(bbox / 256.0), ((df - 1.0) / 2.0 if df > 1.1 else 0.0)


def _gauss_nearest(img: np.ndarray, sigma: float) -> np.ndarray:
    """skimage.filters.gaussian(img, sigma, channel_axis=2, preserve_range=True): separable, mode 'nearest',
    truncate 4 (scipy.ndimage.gaussian_filter1d's radius int(4 sigma + 0.5), uncapped up to the kernel's
    MAX_RADIUS 32); float32 here.  Shares the device kernel's two documented deviations (vge_hmr_front.hip header):
    the blurred patch is rounded to uint8, and bilinear weights are float rather than cv2's fixed point."""
    r = int(4.0 * sigma + 0.5)
    if r > 32:
        raise ValueError(f"gaussian radius {r} > 32 (box too large for the crop kernel)")
    t = np.exp(-0.5 * np.arange(r + 1) ** 2 / sigma ** 2)
    t = (t / (t[0] + 2 * t[1:].sum())).astype(np.float32)
    x = img.astype(np.float32)
    H, W = x.shape[:2]
    out = np.zeros_like(x)
    for dy in range(-r, r + 1):
        ry = np.clip(np.arange(H) + dy, 0, H - 1)
        row = np.zeros_like(x)
        for dx in range(-r, r + 1):
            rx = np.clip(np.arange(W) + dx, 0, W - 1)
            row += t[abs(dx)] * x[ry][:, rx]
        out += t[abs(dy)] * row
    return out


def vitdet_crop(frame_rgb: np.ndarray, box) -> np.ndarray:
    """uint8 [H, W, 3] RGB frame + xyxy box -> uint8 [256, 256, 3] RGB patch (ViTDetDataset.__getitem__ before its
    mean / std normalisation, which patchify applies)."""
    cx, cy, k, sigma = vitdet_geometry(box)
    src = _gauss_nearest(frame_rgb, sigma) if sigma > 0 else frame_rgb.astype(np.float32)
    H, W = frame_rgb.shape[:2]
    f32 = np.float32
    u = np.arange(256, dtype=np.float32)
    sx = f32(cx) + (u - f32(128.0)) * k
    sy = f32(cy) + (u - f32(128.0)) * k
    x0 = np.floor(sx)
    y0 = np.floor(sy)
    fx = (sx - x0)[None, :]
    fy = (sy - y0)[:, None]
    x0 = x0.astype(np.int64)
    y0 = y0.astype(np.int64)
    pad = np.zeros((H + 2, W + 2, 3), np.float32)  # BORDER_CONSTANT 0 around the frame
    pad[1:-1, 1:-1] = src

    def px(yy, xx):
        yy = np.clip(yy + 1, 0, H + 1)
        xx = np.clip(xx + 1, 0, W + 1)
        return pad[yy[:, None], xx[None, :]]

    one = f32(1.0)
    top = (one - fx)[..., None] * px(y0, x0) + fx[..., None] * px(y0, x0 + 1)
    bot = (one - fx)[..., None] * px(y0 + 1, x0) + fx[..., None] * px(y0 + 1, x0 + 1)
    val = (one - fy)[..., None] * top + fy[..., None] * bot
    return np.rint(np.clip(val, 0, 255)).astype(np.uint8)


def single_person_mask(scores: np.ndarray, thresh: float = 0.5) -> np.ndarray:
    """mesh_generator.py:103-111 on the detector's first two NMS-kept persons: exactly one box with score > 0.5."""
    s = np.asarray(scores, np.float32).reshape(-1, 2)
    return (s[:, 0] > thresh) & ~(s[:, 1] > thresh)
