"""Deterministic synthetic inputs in the reference's on-disk layout.

There are no datasets, checkpoints or extractors offline, so every test, fixture and benchmark
runs on data from this generator.  Values are shaped like the real extractor outputs:

* pose / global_orient: valid SO(3) matrices from a per-joint random walk on unit quaternions
  (uniform start, per-frame step ~ N(0, 0.025^2) per component, ~0.05 rad); joint 0 ->
  global_orient [T,1,3,3], joints 1..23 -> pose [T,23,3,3]  (layout of extract_mesh.py:18-43).
  Bit-reproducible on any host CPU (no SIMD transcendental functions).
* betas ~ N(0,1) [T,10];  vit ~ N(0,1) [T,1024]  (token_head.py token_out).
* keypoints ~ U[0,1] [T',120] with ~5% coordinates set to -1 (dwpose_init.py:57-60 marks
  low-score points -1) and an optional T' < T (process_video.py drops frames).

Seeds: real = 1, generated = 2, weights = 3, kp = 4 (mixed with the video index so every clip is
independent of how many other clips are generated).
"""
from __future__ import annotations

import hashlib
import json
import os
from dataclasses import dataclass
from pathlib import Path
from typing import Dict, List, Optional, Sequence

import numpy as np

from .data import ACTION_CLASSES

SEED_REAL, SEED_GEN, SEED_WEIGHTS, SEED_KP = 1, 2, 3, 4
GEN_MODELS = ["Hunyuan", "Opensora_768", "wan21", "RunwayGen4", "Wan2.2"]


def _rodrigues(aa: np.ndarray) -> np.ndarray:
    """axis-angle [...,3] (float64) -> rotation matrices [...,3,3] (float64).  Test helper only: uses
    SIMD sin/cos, so its last bits can differ between host CPUs (never used for fixture inputs)."""
    theta = np.linalg.norm(aa, axis=-1, keepdims=True)
    k = aa / np.maximum(theta, 1e-12)
    kx, ky, kz = k[..., 0], k[..., 1], k[..., 2]
    z = np.zeros_like(kx)
    K = np.stack([np.stack([z, -kz, ky], -1), np.stack([kz, z, -kx], -1),
                  np.stack([-ky, kx, z], -1)], -2)
    s = np.sin(theta)[..., None]
    c = np.cos(theta)[..., None]
    eye = np.broadcast_to(np.eye(3), K.shape)
    return eye + s * K + (1.0 - c) * (K @ K)


def _quat_walk(rng: np.random.Generator, T: int, J: int, step: float = 0.025) -> np.ndarray:
    """Smooth random SO(3) sequences [T,J,3,3] from a random walk on unit quaternions.

    Only element-wise +,-,*,/ and sqrt (IEEE correctly rounded) are used, so the bits are identical on
    every host CPU -- the golden fixtures are regenerated from seeds on the GPU box."""
    def unit(q):
        n = np.sqrt(q[..., 0] * q[..., 0] + q[..., 1] * q[..., 1] + q[..., 2] * q[..., 2] + q[..., 3] * q[..., 3])
        return q / n[..., None]
    q = np.empty((T, J, 4))
    q[0] = unit(rng.normal(0.0, 1.0, size=(J, 4)))
    noise = rng.normal(0.0, step, size=(T, J, 4))
    for t in range(1, T):
        q[t] = unit(q[t - 1] + noise[t])
    w, x, y, z = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    R = np.empty((T, J, 3, 3))
    R[..., 0, 0] = 1 - 2 * (y * y + z * z)
    R[..., 0, 1] = 2 * (x * y - w * z)
    R[..., 0, 2] = 2 * (x * z + w * y)
    R[..., 1, 0] = 2 * (x * y + w * z)
    R[..., 1, 1] = 1 - 2 * (x * x + z * z)
    R[..., 1, 2] = 2 * (y * z - w * x)
    R[..., 2, 0] = 2 * (x * z - w * y)
    R[..., 2, 1] = 2 * (y * z + w * x)
    R[..., 2, 2] = 1 - 2 * (x * x + y * y)
    return R


@dataclass
class SynthClip:
    pose: np.ndarray           # [T,23,3,3] f32
    global_orient: np.ndarray  # [T,1,3,3] f32
    betas: np.ndarray          # [T,10] f32
    vit: np.ndarray            # [T,1024] f32
    keypoints: np.ndarray      # [T',120] f32


def make_clip(seed: int, index: int, T: int, kp_len: Optional[int] = None, vit_dim: int = 1024,
              kp_seed: int = SEED_KP) -> SynthClip:
    rng = np.random.default_rng([seed, index])
    R = _quat_walk(rng, T, 24).astype(np.float32)               # [T,24,3,3]
    betas = rng.normal(0.0, 1.0, size=(T, 10)).astype(np.float32)
    vit = rng.normal(0.0, 1.0, size=(T, vit_dim)).astype(np.float32)
    krng = np.random.default_rng([kp_seed, seed, index])
    Tk = T if kp_len is None else kp_len
    kp = krng.random((Tk, 120), dtype=np.float64).astype(np.float32)
    kp[krng.random((Tk, 120)) < 0.05] = -1.0
    return SynthClip(pose=np.ascontiguousarray(R[:, 1:]), global_orient=np.ascontiguousarray(R[:, :1]),
                     betas=betas, vit=vit, keypoints=kp)


def save_clip_npz(path: Path, clip: SynthClip, meta: Optional[dict] = None) -> None:
    """Same keys and dtypes as extract_mesh.py:35-43 (np.savez_compressed)."""
    path.parent.mkdir(parents=True, exist_ok=True)
    T = clip.pose.shape[0]
    np.savez_compressed(path, pose=clip.pose, betas=clip.betas, global_orient=clip.global_orient,
                        vit=clip.vit, frame_idx=np.arange(T, dtype=np.int32),
                        meta=json.dumps(meta or {}, ensure_ascii=False))


def _hash8(s: str) -> str:
    return hashlib.sha1(s.encode()).hexdigest()[:8]


def generated_name(i: int, classes: Sequence[str] = ACTION_CLASSES) -> str:
    model = GEN_MODELS[i % len(GEN_MODELS)]
    action = classes[(i // len(GEN_MODELS)) % len(classes)]
    nn = i // (len(GEN_MODELS) * len(classes))
    return f"{model}_{action}_{nn:02d}_{_hash8(f'{model}{action}{i}')}"


def write_dataset(root: str, n_real_per_class: int = 5, n_gen: int = 4, T_real: Sequence[int] = (32,),
                  T_gen: Sequence[int] = (32,), kp_short_every: int = 0, classes: Sequence[str] = ACTION_CLASSES,
                  vit_dim: int = 1024) -> Dict[str, str]:
    """Write a synthetic dataset in the reference layout.

    real:      <root>/real/<Class>/v_<Class>_gNN.npz     + <root>/real_kp/<Class>/<stem>/keypoints.npy
    generated: <root>/generated_meshes/<name>.npz        + <root>/generated_kps/<stem>/keypoints.npy
    Lengths cycle through T_real / T_gen; every `kp_short_every`-th clip gets a keypoint file
    5 frames shorter than its mesh sequence (process_video.py drops frames)."""
    root_p = Path(root)
    paths = {k: str(root_p / k) for k in ("real", "real_kp", "generated_meshes", "generated_kps")}
    idx = 0
    for ci, cls in enumerate(classes):
        for j in range(n_real_per_class):
            T = T_real[idx % len(T_real)]
            kp_len = max(1, T - 5) if kp_short_every and idx % kp_short_every == kp_short_every - 1 else None
            clip = make_clip(SEED_REAL, idx, T, kp_len, vit_dim)
            stem = f"v_{cls}_g{j:02d}"
            save_clip_npz(root_p / "real" / cls / f"{stem}.npz", clip, {"video": stem})
            kp_dir = root_p / "real_kp" / cls / stem
            kp_dir.mkdir(parents=True, exist_ok=True)
            np.save(kp_dir / "keypoints.npy", clip.keypoints)
            idx += 1
    for i in range(n_gen):
        T = T_gen[i % len(T_gen)]
        kp_len = max(1, T - 5) if kp_short_every and i % kp_short_every == kp_short_every - 1 else None
        clip = make_clip(SEED_GEN, i, T, kp_len, vit_dim)
        stem = generated_name(i, classes)
        save_clip_npz(root_p / "generated_meshes" / f"{stem}.npz", clip, {"video": stem})
        kp_dir = root_p / "generated_kps" / stem
        kp_dir.mkdir(parents=True, exist_ok=True)
        np.save(kp_dir / "keypoints.npy", clip.keypoints)
    return paths


# ----------------------------------------------------------------------------- weights

def _sinusoidal_pe(d_model: int, max_len: int = 5000) -> np.ndarray:
    """The model.py:9-16 formula (pe[p, 2i] = sin(p / 10000^(2i/d)), pe[p, 2i+1] = cos(...)), evaluated
    with the scalar libm in float64 so the buffer is bit-identical on every host (it is loaded from
    the state_dict, so the reference uses exactly these values too)."""
    import math
    pe = np.zeros((max_len, d_model), np.float64)
    for i in range(0, d_model, 2):
        div = math.exp(i * (-math.log(10000.0) / d_model))
        for p in range(max_len):
            pe[p, i] = math.sin(p * div)
            if i + 1 < d_model:
                pe[p, i + 1] = math.cos(p * div)
    return pe.astype(np.float32)[None]


def make_state_dict(dims_raw: Dict[str, int], dims_diff: Dict[str, int], d_model: int = 256,
                    time_layers: int = 4, ff_mult: int = 4, seed: int = SEED_WEIGHTS,
                    max_len: int = 5000) -> Dict[str, np.ndarray]:
    """Deterministic random weights with exactly the reference state_dict key set
    (model.py:102-148; 241 tensors for the 5-modality model).

    Matrices are U(-1/sqrt(fan_in), 1/sqrt(fan_in)) like torch's default init; norm affines are
    1 + N(0, 0.1) / N(0, 0.1) so the affine paths are exercised; fusion temperature/bias
    ~ N(0, 0.5)."""
    rng = np.random.default_rng(seed)
    sd: Dict[str, np.ndarray] = {}

    def U(shape, fan_in):
        b = 1.0 / np.sqrt(fan_in)
        return rng.uniform(-b, b, size=shape).astype(np.float32)

    def affine(prefix, n):
        sd[prefix + ".weight"] = (1.0 + rng.normal(0, 0.1, n)).astype(np.float32)
        sd[prefix + ".bias"] = rng.normal(0, 0.1, n).astype(np.float32)

    mods = list(dims_raw.keys())
    D = d_model
    for kind, dims in (("state_enc", dims_raw), ("motion_enc", dims_diff)):
        for m in mods:
            if kind == "motion_enc" and dims[m] <= 0:
                continue
            p = f"{kind}.{m}"
            sd[p + ".stem.weight"] = U((D, dims[m], 1), dims[m])
            for i in range(4):
                sd[f"{p}.blocks.{i}.conv1.weight"] = U((D, D, 5), D * 5)
                sd[f"{p}.blocks.{i}.conv2.weight"] = U((D, D, 5), D * 5)
                affine(f"{p}.blocks.{i}.norm", D)
            sd[p + ".proj.weight"] = U((D, D), D)
    M = len(mods)
    sd["fusion.latent"] = rng.normal(0, 1, (1, 1, D)).astype(np.float32)
    sd["fusion.logit_temp"] = rng.normal(0, 0.5, M).astype(np.float32)
    sd["fusion.logit_bias"] = rng.normal(0, 0.5, M).astype(np.float32)
    affine("fusion.q_ln", D)
    affine("fusion.kv_ln", D)
    for w in ("Wq", "Wk", "Wv", "Wo"):
        sd[f"fusion.{w}.weight"] = U((D, D), D)
    sd["cls"] = rng.normal(0, 1, (1, 1, D)).astype(np.float32)
    sd["pos_enc.pe"] = _sinusoidal_pe(D, max_len)
    F = ff_mult * D
    for l in range(time_layers):
        p = f"temporal.layers.{l}"
        sd[p + ".self_attn.in_proj_weight"] = U((3 * D, D), D)
        sd[p + ".self_attn.in_proj_bias"] = rng.normal(0, 0.02, 3 * D).astype(np.float32)
        sd[p + ".self_attn.out_proj.weight"] = U((D, D), D)
        sd[p + ".self_attn.out_proj.bias"] = rng.normal(0, 0.02, D).astype(np.float32)
        sd[p + ".linear1.weight"] = U((F, D), D)
        sd[p + ".linear1.bias"] = rng.normal(0, 0.02, F).astype(np.float32)
        sd[p + ".linear2.weight"] = U((D, F), F)
        sd[p + ".linear2.bias"] = rng.normal(0, 0.02, D).astype(np.float32)
        affine(p + ".norm1", D)
        affine(p + ".norm2", D)
    return sd


DIMS_RAW = {"vit": 1024, "global": 9, "pose": 207, "beta": 10, "kp2d": 120}
DIMS_DIFF = {"vit": 1024, "global": 3, "pose": 69, "beta": 10, "kp2d": 120}


def save_checkpoint(path: str, sd: Dict[str, np.ndarray], d_model: int = 256, time_layers: int = 4,
                    time_heads: int = 8) -> None:
    """{model_state_dict, d_model, time_layers, time_heads, ...} as accepted by eval.py:136-160."""
    import torch
    torch.save({"model_state_dict": {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()},
                "d_model": d_model, "latent_dim": 128, "time_layers": time_layers,
                "time_heads": time_heads, "dropout": 0.1}, path)


def make_hmr_state_dict(cfg, seed: int = SEED_WEIGHTS + 10) -> Dict[str, np.ndarray]:
    """Deterministic random weights for the TokenHMR extractor (vge.hmr.HmrConfig shapes, the upstream
    state_dict key names of include/vge_hmr.h).  No trained weights exist offline, so the extractor is
    measured and parity-checked on these (parity vs upstream TokenHMR unpinned).  Linear weights
    U(-1/sqrt(fan_in), 1/sqrt(fan_in)) (torch's default), biases N(0, 0.02), LayerNorm affines 1 + N(0, 0.1) /
    N(0, 0.1), ViT pos_embed N(0, 0.02) (trunc-normal init), decoder pos_embedding N(0, 1), mean pose = identity
    6D + N(0, 0.1)."""
    rng = np.random.default_rng(seed)
    sd: Dict[str, np.ndarray] = {}

    def U(shape, fan_in):
        b = np.float32(1.0 / np.sqrt(fan_in))
        return (rng.random(size=shape, dtype=np.float32) * (2 * b) - b).astype(np.float32)

    def N(shape, s):
        return (rng.standard_normal(size=shape, dtype=np.float32) * np.float32(s)).astype(np.float32)

    def linear(prefix, n, k, bias=True):
        sd[prefix + ".weight"] = U((n, k), k)
        if bias:
            sd[prefix + ".bias"] = N((n,), 0.02)

    def norm(prefix, n):
        sd[prefix + ".weight"] = (1.0 + N((n,), 0.1)).astype(np.float32)
        sd[prefix + ".bias"] = N((n,), 0.1)

    E, P = cfg.embed_dim, cfg.patch
    sd["backbone.patch_embed.proj.weight"] = U((E, 3, P, P), 3 * P * P)
    sd["backbone.patch_embed.proj.bias"] = N((E,), 0.02)
    sd["backbone.pos_embed"] = N((1, 193, E), 0.02)
    for i in range(cfg.depth):
        b = f"backbone.blocks.{i}."
        norm(b + "norm1", E)
        linear(b + "attn.qkv", 3 * E, E)
        linear(b + "attn.proj", E, E)
        norm(b + "norm2", E)
        linear(b + "mlp.fc1", cfg.mlp_dim, E)
        linear(b + "mlp.fc2", E, cfg.mlp_dim)
    norm("backbone.last_norm", E)
    D, inner = cfg.dec_dim, cfg.dec_heads * cfg.dec_dim_head
    t = "smpl_head.transformer."
    linear(t + "to_token_embedding", D, 1)
    sd[t + "pos_embedding"] = N((1, 1, D), 1.0)
    for l in range(cfg.dec_depth):
        p = f"{t}transformer.layers.{l}."
        norm(p + "0.norm", D)
        linear(p + "0.fn.to_qkv", 3 * inner, D, bias=False)
        linear(p + "0.fn.to_out.0", D, inner)
        norm(p + "1.norm", D)
        linear(p + "1.fn.to_q", inner, D, bias=False)
        linear(p + "1.fn.to_kv", 2 * inner, E, bias=False)
        linear(p + "1.fn.to_out.0", D, inner)
        norm(p + "2.norm", D)
        linear(p + "2.fn.net.0", cfg.dec_mlp, D)
        linear(p + "2.fn.net.3", D, cfg.dec_mlp)
    s = "smpl_head."
    linear(s + "decpose_grot", 6, D)
    linear(s + "decpose_hands", 12, D)
    linear(s + "decshape", 10, D)
    linear(s + "deccam", 3, D)
    linear(s + "decpose.cls", cfg.tok_num * cfg.tok_classes, D)
    sd[s + "decpose.codebook"] = N((cfg.tok_classes, cfg.tok_code_dim), 1.0)
    linear(s + "decpose.dec", 21 * 6, cfg.tok_num * cfg.tok_code_dim)
    ident = np.tile(np.array([1, 0, 0, 0, 1, 0], np.float32), 24)
    sd[s + "init_body_pose"] = (ident + N((144,), 0.1))[None]
    sd[s + "init_betas"] = N((1, 10), 0.5)
    sd[s + "init_cam"] = np.array([[0.9, 0.0, 0.0]], np.float32)
    return sd


def make_frames(seed: int, n_frames: int, h: int = 256, w: int = 256) -> np.ndarray:
    """uint8 RGB person-crop frames [F, h, w, 3]: a per-clip random low-frequency image drifting by a few
    pixels per frame plus pixel noise (shape of ViTDetDataset's 256x256 crops)."""
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, size=(h // 8 + 8, w // 8 + 8, 3), dtype=np.uint8)
    big = np.kron(base, np.ones((8, 8, 1), np.uint8))
    out = np.empty((n_frames, h, w, 3), np.uint8)
    for f in range(n_frames):
        dy, dx = f % 8, (2 * f) % 8
        noise = rng.integers(-12, 13, size=(h, w, 3))
        out[f] = np.clip(big[dy:dy + h, dx:dx + w].astype(np.int32) + noise, 0, 255).astype(np.uint8)
    return out


def make_rtmpose_state_dict(cfg, seed: int = SEED_WEIGHTS + 20, gain: float = 1.0) -> Dict[str, np.ndarray]:
    """Deterministic random weights for the DWPose whole-body pose model (vge.dwpose.RtmposeConfig shapes;
    mmpose RTMPose state_dict keys: CSPNeXt backbone.stem / backbone.stage<i>, RTMCCHead head.*).  No trained
    weights exist offline (DWPose ships dw-ll_ucoco_384.onnx by download), so the model is measured and
    parity-checked on these (parity vs the upstream ONNX unpinned).  Conv weights N(0, 2/fan_in) (He init, so
    SiLU activations stay O(1) through the 40-odd layers), BatchNorm gamma 1 + N(0, 0.1), beta / running mean
    N(0, 0.1), running var U(0.5, 1.5); head Linears U(-1/sqrt(fan_in), 1/sqrt(fan_in)); GAU gamma/beta
    N(0, 1) / N(0, 0.1) scaled to keep the squared-ReLU kernel O(1)."""
    rng = np.random.default_rng(seed)
    sd: Dict[str, np.ndarray] = {}

    def N(shape, s):
        return (rng.standard_normal(size=shape, dtype=np.float32) * np.float32(s)).astype(np.float32)

    def U(shape, fan_in):
        b = np.float32(1.0 / np.sqrt(fan_in))
        return (rng.random(size=shape, dtype=np.float32) * (2 * b) - b).astype(np.float32)

    def convmod(prefix, cin, cout, k, groups=1):
        fan = (cin // groups) * k * k
        sd[prefix + ".conv.weight"] = N((cout, cin // groups, k, k), np.sqrt(gain / fan))
        sd[prefix + ".bn.weight"] = (1.0 + N((cout,), 0.1)).astype(np.float32)
        sd[prefix + ".bn.bias"] = N((cout,), 0.1)
        sd[prefix + ".bn.running_mean"] = N((cout,), 0.1)
        sd[prefix + ".bn.running_var"] = (0.5 + rng.random(size=(cout,), dtype=np.float32)).astype(np.float32)

    def csp(prefix, cin, cout, n, add_identity):
        mid = cout // 2
        convmod(prefix + ".main_conv", cin, mid, 1)
        convmod(prefix + ".short_conv", cin, mid, 1)
        convmod(prefix + ".final_conv", 2 * mid, cout, 1)
        for b in range(n):
            p = f"{prefix}.blocks.{b}"
            convmod(p + ".conv1", mid, mid, 3)
            convmod(p + ".conv2.depthwise_conv", mid, mid, 5, groups=mid)
            convmod(p + ".conv2.pointwise_conv", mid, mid, 1)
        sd[prefix + ".attention.fc.weight"] = N((2 * mid, 2 * mid, 1, 1), np.sqrt(1.0 / (2 * mid)))
        sd[prefix + ".attention.fc.bias"] = N((2 * mid,), 0.1)

    s0 = cfg.stem_ch
    convmod("backbone.stem.0", 3, s0 // 2, 3)
    convmod("backbone.stem.1", s0 // 2, s0 // 2, 3)
    convmod("backbone.stem.2", s0 // 2, s0, 3)
    cin = s0
    for i, (cout, n) in enumerate(zip(cfg.stage_ch, cfg.stage_blocks)):
        st = f"backbone.stage{i + 1}"
        convmod(st + ".0", cin, cout, 3)
        j = 1
        if i == 3:  # SPPBottleneck(5, 9, 13) on the last stage
            convmod(st + ".1.conv1", cout, cout // 2, 1)
            convmod(st + ".1.conv2", (cout // 2) * 4, cout, 1)
            j = 2
        csp(f"{st}.{j}", cout, cout, n, add_identity=(i < 3))
        cin = cout
    K, hw = cfg.keypoints, (cfg.in_h // 32) * (cfg.in_w // 32)
    fk = cfg.final_k
    sd["head.final_layer.weight"] = N((K, cin, fk, fk), np.sqrt(1.0 / (cin * fk * fk)))
    sd["head.final_layer.bias"] = N((K,), 0.1)
    sd["head.mlp.0.g"] = np.ones((1,), np.float32)
    sd["head.mlp.1.weight"] = U((cfg.gau_hidden, hw), hw)
    H, S, E = cfg.gau_hidden, cfg.gau_s, cfg.gau_e
    sd["head.gau.uv.weight"] = U((2 * E + S, H), H)
    sd["head.gau.gamma"] = N((2, S), 1.0)
    sd["head.gau.beta"] = N((2, S), 0.1)
    sd["head.gau.o.weight"] = U((H, E), E)
    sd["head.gau.ln.g"] = np.ones((1,), np.float32)
    sd["head.gau.res_scale.scale"] = (1.0 + N((H,), 0.1)).astype(np.float32)
    sd["head.cls_x.weight"] = U((cfg.in_w * cfg.split, H), H)
    sd["head.cls_y.weight"] = U((cfg.in_h * cfg.split, H), H)
    return sd


def make_yolox_state_dict(cfg, seed: int = SEED_WEIGHTS + 30, gain: float = 1.0) -> Dict[str, np.ndarray]:
    """Deterministic random weights for DWPose's YOLOX person detector (vge.dwpose.YoloxConfig shapes; the
    official YOLOX state_dict keys: backbone.backbone.{stem,dark2..dark5}, backbone.{lateral_conv0, C3_p4,
    reduce_conv1, C3_p3, bu_conv2, C3_n3, bu_conv1, C3_n4}, head.{stems, cls_convs, reg_convs, cls_preds,
    reg_preds, obj_preds}).  yolox_l.onnx is a download (no weights offline): parity vs upstream unpinned.
    BaseConv weights N(0, gain/fan_in) (residual-branch 3x3 convs 0.1 gain/fan_in, so the 9-block CSP stages
    stay O(1)), BatchNorm as in make_rtmpose_state_dict; prediction convs small, so sigmoid scores spread
    around the 0.1 / 0.3 thresholds."""
    rng = np.random.default_rng(seed)
    sd: Dict[str, np.ndarray] = {}

    def N(shape, s):
        return (rng.standard_normal(size=shape, dtype=np.float32) * np.float32(s)).astype(np.float32)

    def base(prefix, cin, cout, k, g=1.0):
        sd[prefix + ".conv.weight"] = N((cout, cin, k, k), np.sqrt(g * gain / (cin * k * k)))
        sd[prefix + ".bn.weight"] = (1.0 + N((cout,), 0.1)).astype(np.float32)
        sd[prefix + ".bn.bias"] = N((cout,), 0.1)
        sd[prefix + ".bn.running_mean"] = N((cout,), 0.1)
        sd[prefix + ".bn.running_var"] = (0.5 + rng.random(size=(cout,), dtype=np.float32)).astype(np.float32)

    def csp(prefix, cin, cout, n, shortcut):
        hid = cout // 2
        base(prefix + ".conv1", cin, hid, 1)
        base(prefix + ".conv2", cin, hid, 1)
        base(prefix + ".conv3", 2 * hid, cout, 1)
        for i in range(n):
            base(f"{prefix}.m.{i}.conv1", hid, hid, 1)
            base(f"{prefix}.m.{i}.conv2", hid, hid, 3, 0.1 if shortcut else 1.0)  # small residual branches

    w0, d = cfg.width, cfg.depth
    bb = "backbone.backbone."
    base(bb + "stem.conv", 12, w0, 3)
    base(bb + "dark2.0", w0, 2 * w0, 3)
    csp(bb + "dark2.1", 2 * w0, 2 * w0, d, True)
    base(bb + "dark3.0", 2 * w0, 4 * w0, 3)
    csp(bb + "dark3.1", 4 * w0, 4 * w0, 3 * d, True)
    base(bb + "dark4.0", 4 * w0, 8 * w0, 3)
    csp(bb + "dark4.1", 8 * w0, 8 * w0, 3 * d, True)
    base(bb + "dark5.0", 8 * w0, 16 * w0, 3)
    base(bb + "dark5.1.conv1", 16 * w0, 8 * w0, 1)
    base(bb + "dark5.1.conv2", 32 * w0, 16 * w0, 1)
    csp(bb + "dark5.2", 16 * w0, 16 * w0, d, False)
    c3, c4, c5 = 4 * w0, 8 * w0, 16 * w0
    base("backbone.lateral_conv0", c5, c4, 1)
    csp("backbone.C3_p4", 2 * c4, c4, d, False)
    base("backbone.reduce_conv1", c4, c3, 1)
    csp("backbone.C3_p3", 2 * c3, c3, d, False)
    base("backbone.bu_conv2", c3, c3, 3)
    csp("backbone.C3_n3", 2 * c3, c4, d, False)
    base("backbone.bu_conv1", c4, c4, 3)
    csp("backbone.C3_n4", 2 * c4, c5, d, False)
    hc = cfg.head_ch
    for k, cin in enumerate((c3, c4, c5)):
        base(f"head.stems.{k}", cin, hc, 1)
        for br in ("cls_convs", "reg_convs"):
            base(f"head.{br}.{k}.0", hc, hc, 3)
            base(f"head.{br}.{k}.1", hc, hc, 3)
        sd[f"head.cls_preds.{k}.weight"] = N((cfg.num_classes, hc, 1, 1), 0.01 * np.sqrt(hc))
        sd[f"head.cls_preds.{k}.bias"] = N((cfg.num_classes,), 0.5)
        sd[f"head.reg_preds.{k}.weight"] = N((4, hc, 1, 1), 0.3 / np.sqrt(hc))
        sd[f"head.reg_preds.{k}.bias"] = N((4,), 0.2)
        sd[f"head.obj_preds.{k}.weight"] = N((1, hc, 1, 1), 0.01 * np.sqrt(hc))
        sd[f"head.obj_preds.{k}.bias"] = N((1,), 0.5)
    return sd


# The e2e bench's person detector (TokenHMR's single-person gate, mesh_generator.py:103-117, and DWPose's boxes).
# With make_yolox_state_dict's weights every synthetic frame has several person boxes above 0.5, so the gate would
# reject every video.  These weights differ from it in the prediction biases only: the person class probability is
# saturated (score = objectness), one common shift of the objectness logits (the anchors' ranking, hence which boxes
# NMS keeps, is unchanged) puts the 0.5 threshold between the first and the second kept box of as many pool frames
# as possible, and box sizes are person-like (about GATE_BOX_STRIDES (w, h) strides).  GATE_OBJ_SHIFT is measured on
# make_frame_pool's frames on the GPU (the detector runs in bf16 there; it was the round-4 gate, whose calibration
# script went with it -- the current gate is the Faster R-CNN, tools/frcnn_gate_calib.py); VGE_GATE_OBJ_SHIFT overrides
# it for a calibration run.
GATE_OBJ_SHIFT = float(os.environ.get("VGE_GATE_OBJ_SHIFT", "3.911"))
GATE_BOX_STRIDES = (6.0, 60.0)


def make_gate_detector_state_dict(cfg, obj_shift: float = None, box_strides=GATE_BOX_STRIDES):
    sd = make_yolox_state_dict(cfg)
    shift = GATE_OBJ_SHIFT if obj_shift is None else obj_shift
    for k in range(3):
        sd[f"head.cls_preds.{k}.bias"][0] = np.float32(30.0)
        sd[f"head.obj_preds.{k}.bias"] = (sd[f"head.obj_preds.{k}.bias"] - np.float32(shift)).astype(np.float32)
        sd[f"head.reg_preds.{k}.bias"][2:] += np.log(np.asarray(box_strides, np.float32))
    return sd


def make_frame_pool(seed: int, n_frames: int, per_scene: int = 4, h: int = 256, w: int = 256) -> np.ndarray:
    """uint8 RGB frames [n_frames, h, w, 3] from n_frames / per_scene independent make_frames scenes: the pool the
    e2e bench draws its clips' frames from, by what the detector finds in each."""
    scenes = [make_frames(seed + i, per_scene, h, w) for i in range(-(-n_frames // per_scene))]
    return np.concatenate(scenes, 0)[:n_frames]


def make_frcnn_state_dict(cfg, seed: int = SEED_WEIGHTS + 40, cls_gain: float = 4.0) -> Dict[str, np.ndarray]:
    """Deterministic random weights for TokenHMR's gate detector, detectron2's Faster R-CNN X101-32x8d-FPN
    (vge.frcnn.FrcnnConfig shapes, detectron2 state_dict keys).  The model-zoo weights are a download (none offline):
    parity vs detectron2 is unpinned.  Convs He-initialised N(0, 2 / fan_in) with the bottleneck's last conv at 0.02 /
    fan_in (the 23-block res4 stream stays O(1)), FPN convs 0.25 / 0.5 over fan_in, FrozenBN weight 1 + N(0, 0.1), bias / running mean N(0, 0.1),
    running var U(0.5, 1.5); FPN / RPN / fc biases N(0, 0.1); objectness logits O(1) (no flat ties among the top-k);
    box deltas ~0.1; cls_score N(0, cls_gain^2 / 1024) + N(0, 1) biases, so the softmax over 81 classes is peaked and
    most proposals carry one or two classes above the 0.25 threshold (every class-aware path runs)."""
    rng = np.random.default_rng(seed)
    sd: Dict[str, np.ndarray] = {}

    def N(shape, s):
        return (rng.standard_normal(size=shape, dtype=np.float32) * np.float32(s)).astype(np.float32)

    def conv_bn(name, cin, cout, k, groups=1, gain=2.0):
        fan = (cin // groups) * k * k
        sd[name + ".weight"] = N((cout, cin // groups, k, k), np.sqrt(gain / fan))
        sd[name + ".norm.weight"] = (1.0 + N((cout,), 0.1)).astype(np.float32)
        sd[name + ".norm.bias"] = N((cout,), 0.1)
        sd[name + ".norm.running_mean"] = N((cout,), 0.1)
        sd[name + ".norm.running_var"] = (0.5 + rng.random(size=(cout,), dtype=np.float32)).astype(np.float32)

    def conv_b(name, cin, cout, k, gain=1.0, bias=0.1):
        sd[name + ".weight"] = N((cout, cin, k, k), np.sqrt(gain / (cin * k * k)))
        sd[name + ".bias"] = N((cout,), bias)

    def linear(name, cin, cout, std, bias=0.1):
        sd[name + ".weight"] = N((cout, cin), std)
        sd[name + ".bias"] = N((cout,), bias)

    bb = "backbone.bottom_up."
    conv_bn(bb + "stem.conv1", 3, cfg.stem_ch, 7)
    blocks = {50: (3, 4, 6, 3), 101: (3, 4, 23, 3), 152: (3, 8, 36, 3)}[cfg.depth]
    cin, width, out = cfg.stem_ch, cfg.groups * cfg.width_per_group, cfg.res2_ch
    for s, nb in enumerate(blocks):
        for b in range(nb):
            p = f"{bb}res{s + 2}.{b}"
            if b == 0:
                conv_bn(p + ".shortcut", cin, out, 1, gain=1.0)
            conv_bn(p + ".conv1", cin if b == 0 else out, width, 1)
            conv_bn(p + ".conv2", width, width, 3, groups=cfg.groups)
            conv_bn(p + ".conv3", width, out, 1, gain=0.02)
        cin, width, out = out, width * 2, out * 2
    F = cfg.fpn_ch
    for l in range(4):
        conv_b(f"backbone.fpn_lateral{l + 2}", cfg.res2_ch << l, F, 1, gain=0.25)
        conv_b(f"backbone.fpn_output{l + 2}", F, F, 3, gain=0.5)
    conv_b("proposal_generator.rpn_head.conv", F, F, 3, gain=2.0)
    conv_b("proposal_generator.rpn_head.objectness_logits", F, 3, 1, gain=1.0, bias=0.5)
    conv_b("proposal_generator.rpn_head.anchor_deltas", F, 12, 1, gain=0.01, bias=0.0)
    linear("roi_heads.box_head.fc1", F * cfg.pool * cfg.pool, cfg.fc_dim, np.sqrt(2.0 / (F * cfg.pool * cfg.pool)))
    linear("roi_heads.box_head.fc2", cfg.fc_dim, cfg.fc_dim, np.sqrt(2.0 / cfg.fc_dim))
    linear("roi_heads.box_predictor.cls_score", cfg.fc_dim, cfg.num_classes + 1, cls_gain / np.sqrt(cfg.fc_dim), 1.0)
    linear("roi_heads.box_predictor.bbox_pred", cfg.fc_dim, 4 * cfg.num_classes, 0.1 / np.sqrt(cfg.fc_dim), 0.0)
    return sd


# The e2e bench's gate detector (mesh_generator.py:103-117 with the reference's Faster R-CNN).  With
# make_frcnn_state_dict's weights most frames have several person instances above 0.5, so the gate would reject every
# video.  These weights differ in the predictor's class biases only: classes 1..79 at -20 (never above 0.25), so a
# proposal's person probability is sigmoid(person logit - background logit); one common background bias (the person
# logits' ranking, hence which boxes the class-aware NMS keeps, is unchanged) puts the 0.5 threshold between the first
# and second kept person instance of as many pool frames as possible.  GATE_FRCNN_BG is measured on make_frame_pool's
# frames by tools/frcnn_gate_calib.py on the GPU; VGE_GATE_FRCNN_BG overrides it for a calibration run.
GATE_FRCNN_BG = float(os.environ.get("VGE_GATE_FRCNN_BG", "-0.5007"))


def make_gate_frcnn_state_dict(cfg, bg: float = None) -> Dict[str, np.ndarray]:
    sd = make_frcnn_state_dict(cfg)
    b = sd["roi_heads.box_predictor.cls_score.bias"]
    b[0] = np.float32(0.0)
    b[1:cfg.num_classes] = np.float32(-20.0)
    b[cfg.num_classes] = np.float32(GATE_FRCNN_BG if bg is None else bg)
    return sd
