"""ORACLE (test infrastructure only): numpy-float32 restatement of the reference featurisation.

Follows /root/reference/utils.py op for op:
  _log_so3              utils.py:130-140
  _vit_delta            utils.py:142-147
  _betas_delta          utils.py:161-163
  _rotmat_delta         utils.py:165-174
  _procrustes_kp_delta  utils.py:177-217 (2x2 SVD through oracle.lapack2x2, LAPACK signs)
  slice_or_pad          utils.py:366-381
  featurize_window      utils.py:383-516 (WindowDataset._try_one, z-norm eps 1e-6 at 472-494)
  accumulate_stats / finalize_stats   utils.py:589-593, 595-801 (float64 sums, eps 1e-6 in std)
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np

from .lapack2x2 import sgesdd_2x2

f32 = np.float32

# Column layout of feats [T, 2596] (utils.py:496-514; dims train.py:29-47)
RAW_ORDER = ("vit", "global", "pose", "beta", "kp2d")
RAW_DIMS = {"vit": 1024, "global": 9, "pose": 207, "beta": 10, "kp2d": 120}
DIFF_DIMS = {"vit": 1024, "global": 3, "pose": 69, "beta": 10, "kp2d": 120}


def _mm3(A, B):
    """Batched 3x3 product A @ B in float32, k summed left to right."""
    out = np.empty(np.broadcast_shapes(A.shape, B.shape), f32)
    for i in range(3):
        for j in range(3):
            out[..., i, j] = ((A[..., i, 0] * B[..., 0, j]).astype(f32) + (A[..., i, 1] * B[..., 1, j]).astype(f32)
                              ).astype(f32) + (A[..., i, 2] * B[..., 2, j]).astype(f32)
    return out


def log_so3(R: np.ndarray) -> np.ndarray:
    """utils.py:130-140."""
    R = R.astype(f32)
    tr = ((R[..., 0, 0] + R[..., 1, 1]).astype(f32) + R[..., 2, 2]).astype(f32)
    tr = np.clip(tr, f32(-1 + 1e-6), f32(3 - 1e-6)).astype(f32)
    theta = np.arccos(((tr - f32(1)) / f32(2)).astype(f32)).astype(f32)
    denom = np.maximum((f32(2) * np.sin(theta)).astype(f32), f32(1e-6)).astype(f32)
    v = np.stack([R[..., 2, 1] - R[..., 1, 2], R[..., 0, 2] - R[..., 2, 0], R[..., 1, 0] - R[..., 0, 1]],
                 axis=-1).astype(f32) / denom[..., None]
    return (theta[..., None] * v.astype(f32)).astype(f32)


def rotmat_delta(R: np.ndarray) -> np.ndarray:
    """utils.py:165-174: Rrel = R_{t-1}^T R_t with R_{-1} = R_0; returns log map [T, ..., 3]."""
    Rp = np.concatenate([R[:1], R[:-1]], axis=0)
    return log_so3(_mm3(np.swapaxes(Rp, -1, -2), R))


def vit_delta(vit: np.ndarray) -> np.ndarray:
    """utils.py:142-147 (F.normalize eps 1e-12)."""
    v = vit.astype(f32)
    n = np.sqrt((v.astype(np.float64) ** 2).sum(-1)).astype(f32)
    v = (v / np.maximum(n, f32(1e-12))[:, None]).astype(f32)
    vp = np.concatenate([v[:1], v[:-1]], axis=0)
    return (v - vp).astype(f32)


def betas_delta(b: np.ndarray) -> np.ndarray:
    """utils.py:161-163."""
    return (b - np.concatenate([b[:1], b[:-1]], axis=0)).astype(f32)


def procrustes_kp_delta(kp: np.ndarray, eps: float = 1e-6) -> np.ndarray:
    """utils.py:177-217: centre, Frobenius-scale, then per consecutive pair H = X^T Y,
    (U,S,Vh) = svd(H) [LAPACK signs], R = Vh U^T (flip Vh[:, -1] if det R < 0), delta = Y - X R."""
    T = kp.shape[0]
    pts = kp.reshape(T, -1, 2).astype(f32)
    mean = (pts.astype(np.float64).sum(1, keepdims=True) / pts.shape[1]).astype(f32)
    pc = (pts - mean).astype(f32)
    s = np.sqrt((pc.astype(np.float64) ** 2).sum(axis=(1, 2), keepdims=True)).astype(f32)
    pn = (pc / np.maximum(s, f32(eps))).astype(f32)
    deltas = np.zeros_like(pn)
    if T > 1:
        X = pn[:-1]
        Y = pn[1:]
        H = np.einsum("nki,nkj->nij", X.astype(np.float64), Y.astype(np.float64)).astype(f32)
        U, _, Vh = sgesdd_2x2(H)
        UT = np.swapaxes(U, -1, -2)
        R = np.einsum("nij,njk->nik", Vh.astype(np.float64), UT.astype(np.float64)).astype(f32)
        det = (R[:, 0, 0].astype(np.float64) * R[:, 1, 1] - R[:, 0, 1].astype(np.float64) * R[:, 1, 0])
        neg = det < 0
        Vh2 = Vh.copy()
        Vh2[:, :, -1] *= -1
        R2 = np.einsum("nij,njk->nik", Vh2.astype(np.float64), UT.astype(np.float64)).astype(f32)
        R = np.where(neg[:, None, None], R2, R)
        Xa = np.einsum("nki,nij->nkj", X.astype(np.float64), R.astype(np.float64)).astype(f32)
        deltas[1:] = (Y - Xa).astype(f32)
    return deltas.reshape(T, -1)


def slice_or_pad(arr: np.ndarray, start: int, T: int) -> np.ndarray:
    """utils.py:366-381 (nearest-repeat padding)."""
    n = arr.shape[0]
    if start < 0 or start >= n:
        idx = 0 if start < 0 else n - 1
        return np.repeat(arr[idx:idx + 1], T, axis=0)
    if start + T <= n:
        return arr[start:start + T]
    tail = arr[start:]
    pad = np.repeat(arr[-1:], T - tail.shape[0], axis=0)
    return np.concatenate([tail, pad], axis=0)


@dataclass
class Stats:
    """ModalityStats (utils.py:570-586) restricted to the 5 live modalities; float32 arrays."""
    mean_raw: Dict[str, np.ndarray]
    std_raw: Dict[str, np.ndarray]
    mean_diff: Dict[str, np.ndarray]
    std_diff: Dict[str, np.ndarray]
    has_kp: bool = True

    def concat(self):
        """(mean[2596], std[2596]) in feats column order."""
        mods = [m for m in RAW_ORDER if self.has_kp or m != "kp2d"]
        mean = np.concatenate([self.mean_raw[m] for m in mods] + [self.mean_diff[m] for m in mods])
        std = np.concatenate([self.std_raw[m] for m in mods] + [self.std_diff[m] for m in mods])
        return mean.astype(f32), std.astype(f32)


def frame_features(pose, gori, betas, vit, kp):
    """Un-normalised raw and diff parts for one (already sliced) sequence.
    Returns dict name -> (raw [T,d], diff [T,d']) following utils.py:396-470."""
    T = pose.shape[0]
    out = {
        "vit": (vit.astype(f32), vit_delta(vit)),
        "global": (gori.reshape(T, -1).astype(f32), rotmat_delta(gori.astype(f32)).reshape(T, -1)),
        "pose": (pose.reshape(T, -1).astype(f32), rotmat_delta(pose.astype(f32)).reshape(T, -1)),
        "beta": (betas.astype(f32), betas_delta(betas.astype(f32))),
    }
    if kp is not None:
        out["kp2d"] = (kp.astype(f32), procrustes_kp_delta(kp))
    return out


def featurize_window(pose, gori, betas, vit, kp, start: int, stats: Optional[Stats], clip_len: int = 32):
    """WindowDataset._try_one (utils.py:383-516) for one (video, start) window -> feats [T, D]."""
    pw = slice_or_pad(pose, start, clip_len)
    gw = slice_or_pad(gori, start, clip_len)
    bw = slice_or_pad(betas, start, clip_len)
    vw = slice_or_pad(vit, start, clip_len)
    kw = slice_or_pad(kp, start, clip_len) if kp is not None else None
    parts = frame_features(pw, gw, bw, vw, kw)
    mods = [m for m in RAW_ORDER if m in parts]
    eps = f32(1e-6)
    raws, diffs = [], []
    for m in mods:
        r, d = parts[m]
        if stats is not None:
            r = ((r - stats.mean_raw[m]).astype(f32) / (stats.std_raw[m] + eps).astype(f32)).astype(f32)
            d = ((d - stats.mean_diff[m]).astype(f32) / (stats.std_diff[m] + eps).astype(f32)).astype(f32)
        raws.append(r)
        diffs.append(d)
    return np.concatenate(raws + diffs, axis=-1).astype(f32)


class StatsAccumulator:
    """compute_stats_from_npz (utils.py:595-801): per-dim float64 sum / sum of squares over all
    frames of the real-train videos (diffs on the full sequence), n = frame counts."""

    def __init__(self):
        self.s: Dict[str, np.ndarray] = {}
        self.ss: Dict[str, np.ndarray] = {}
        self.n: Dict[str, int] = {}

    def _upd(self, key, X):
        X = X.astype(f32)
        if key not in self.s:
            self.s[key] = np.zeros(X.shape[1], np.float64)
            self.ss[key] = np.zeros(X.shape[1], np.float64)
            self.n[key] = 0
        self.s[key] += X.sum(axis=0, dtype=np.float64)
        self.ss[key] += (X.astype(np.float64) ** 2).sum(axis=0)
        self.n[key] += X.shape[0]

    def add_video(self, pose, gori, betas, vit, kp=None):
        parts = frame_features(pose, gori, betas, vit, kp)
        for m, (r, d) in parts.items():
            self._upd(("raw", m), r)
            self._upd(("diff", m), d)

    def finalize(self, eps: float = 1e-6) -> Stats:
        def fin(key):
            n = max(1, self.n[key])
            mean = self.s[key] / n
            var = self.ss[key] / n - mean ** 2
            std = np.sqrt(np.maximum(var, 0.0) + eps)
            return mean.astype(f32), std.astype(f32)
        st = Stats({}, {}, {}, {}, has_kp=("raw", "kp2d") in self.n and self.n[("raw", "kp2d")] > 0)
        for m in RAW_ORDER:
            if ("raw", m) not in self.n:
                continue
            st.mean_raw[m], st.std_raw[m] = fin(("raw", m))
            st.mean_diff[m], st.std_diff[m] = fin(("diff", m))
        return st
