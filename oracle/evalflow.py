"""ORACLE (test infrastructure only): CPU restatement of the reference scoring driver.

Restates /root/reference/eval.py:350-454 with the oracle featuriser and encoder:
  dataset scan / split          utils.py:229-341 (sorted class dirs, random.Random(seed) shuffle)
  stats                         utils.py:595-801 (float64 sums over full real-train videos)
  centroids                     eval.py:260-286 + utils.py:1018-1045 (index_add_ in window order)
  generated windows             eval.py:48-101 + utils.py:888-911
  extract_window_features       eval.py:168-206 (batches of 32)
  TC / AC                       eval.py:209-257
  result JSON                   eval.py:439-451
It is also the CPU baseline timed by bench.py (kind "port"): DataLoader workers featurise,
torch-fp32 CPU encoder, exactly the reference's work split.
"""
from __future__ import annotations

import os
import random
import time
from collections import defaultdict
from pathlib import Path
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from .encoder import OracleEncoder
from .featurize import StatsAccumulator, featurize_window

ACTION_CLASSES = ["BodyWeightSquats", "HulaHoop", "JumpingJack", "PullUps", "PushUps", "Shotput",
                  "SoccerJuggling", "TennisSwing", "ThrowDiscus", "WallPushups"]


def canon(name: str) -> str:
    for c in ACTION_CLASSES:
        if name.lower() == c.lower():
            return c
    return {"soccerjuggling": "SoccerJuggling", "tennisswing": "TennisSwing"}.get(name.lower(), name)


def scan_real(root: str) -> Dict[str, List[Tuple[str, str, int]]]:
    """class -> [(name, path, T)] in scan order (utils.py:268-295)."""
    out: Dict[str, List[Tuple[str, str, int]]] = {}
    for cls in sorted(d for d in os.listdir(root) if os.path.isdir(os.path.join(root, d))):
        if cls not in ACTION_CLASSES:
            continue
        for f in sorted(os.listdir(os.path.join(root, cls))):
            if f.endswith(".npz"):
                p = os.path.join(root, cls, f)
                with np.load(p) as z:
                    out.setdefault(cls, []).append((f, p, int(z["pose"].shape[0])))
    return out


def split(class_items, ratio=0.8, seed=1337):
    rng = random.Random(seed)
    train = []
    for cls, vids in class_items.items():
        v = vids[:]
        rng.shuffle(v)
        n = len(v)
        k = max(1, min(n - 1, int(round(n * ratio))))
        train.extend((cls,) + x for x in v[:k])
    return train


def kp_path(kdir, cls, stem):
    if "SAVE_GEN" in kdir or "SAVE_NEW" in kdir or "generated_kps" in kdir:
        return os.path.join(kdir, stem, "keypoints.npy")
    return os.path.join(kdir, cls, stem, "keypoints.npy")


def load(path, kdir, cls, require_kp=True):
    with np.load(path) as z:
        arrs = [np.asarray(z[k], np.float32) for k in ("pose", "global_orient", "betas", "vit")]
    stem = os.path.splitext(os.path.basename(path))[0]
    kp = None
    if kdir is not None:
        p = kp_path(kdir, cls, stem)
        if os.path.exists(p):
            kp = np.load(p).astype(np.float32)
        elif require_kp:
            raise FileNotFoundError(p)
    return arrs + [kp]


def compute_stats(train, kdir):
    acc = StatsAccumulator()
    for cls, name, path, T in train:
        pose, gori, betas, vit, kp = load(path, kdir, cls, require_kp=False)
        acc.add_video(pose, gori, betas, vit, kp)
    return acc.finalize()


def windows_for(T, clip_len=32, stride=8):
    if T < clip_len:
        return [0]
    return list(range(0, T - clip_len + 1, stride))


class _WinDS(torch.utils.data.Dataset):
    def __init__(self, samples, kdir, stats):
        self.samples, self.kdir, self.stats = samples, kdir, stats

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, i):
        cls, name, path, s = self.samples[i]
        pose, gori, betas, vit, kp = load(path, self.kdir, cls)
        return torch.from_numpy(featurize_window(pose, gori, betas, vit, kp, s, self.stats)), cls, name


def _collate(b):
    f, c, n = zip(*b)
    return torch.stack(f), list(c), list(n)


def encode_samples(enc, samples, kdir, stats, batch_size=32, workers=0):
    dl = torch.utils.data.DataLoader(_WinDS(samples, kdir, stats), batch_size=batch_size, shuffle=False,
                                     num_workers=workers, collate_fn=_collate)
    seqs, frames, clss, names = [], [], [], []
    for feats, c, n in dl:
        s, fe, _ = enc.forward(feats)
        seqs.append(s)
        frames.append(fe)
        clss += c
        names += n
    return torch.cat(seqs), torch.cat(frames), clss, names


def centroids(enc, train, kdir, stats, label_dict):
    samples = [(cls, name, path, s) for cls, name, path, T in train if T > 0 for s in windows_for(T)]
    seq, _, clss, _ = encode_samples(enc, samples, kdir, stats, batch_size=64)
    C = len(label_dict)
    sums = torch.zeros(C, seq.shape[1])
    counts = torch.zeros(C)
    y = torch.as_tensor([label_dict[c] for c in clss], dtype=torch.long)
    sums.index_add_(0, y, seq)
    counts.index_add_(0, y, torch.ones_like(y, dtype=torch.float32))
    return F.normalize(sums / counts.clamp_min(1.0).unsqueeze(1), dim=-1), counts


def scan_generated(gdir):
    items = []
    for p in sorted(Path(gdir).glob("*.npz")):
        parts = p.stem.split("_")
        cls = None
        for part in parts:
            if canon(part) in ACTION_CLASSES:
                cls = canon(part)
                break
        if cls is None:
            for part in parts:
                if part[0].isupper() and not part.isdigit() and len(part) > 3 and part.lower() not in ("videos", "npz"):
                    cls = canon(part)
                    break
        cls = cls or "Unknown"
        with np.load(p) as z:
            T = int(z["pose"].shape[0])
        items.append((cls, p.name, str(p), T))
    # NpzVideoDataset regroups items by class in first-appearance order (utils.py:241-253)
    groups: Dict[str, list] = {}
    for it in items:
        groups.setdefault(it[0], []).append(it)
    return [it for g in groups.values() for it in g]


def tc_scores(frame_embeds, vid_names):
    per = defaultdict(list)
    for i, v in enumerate(vid_names):
        f = frame_embeds[i][1:]
        if f.shape[0] < 2:
            continue
        per[os.path.splitext(v)[0]].append(float((f[1:] - f[:-1]).pow(2).sum(-1).sqrt().mean().item()))
    return {k: float(np.mean(v)) for k, v in per.items()}


def ac_scores(seq, cls_names, vid_names, cents, label_dict):
    emb = defaultdict(list)
    vcls = {}
    for i, v in enumerate(vid_names):
        k = os.path.splitext(v)[0]
        emb[k].append(seq[i])
        vcls[k] = canon(cls_names[i])
    out = {}
    for k, e in emb.items():
        c = vcls[k]
        if c not in label_dict or label_dict[c] >= len(cents):
            continue
        z = F.normalize(torch.stack(e).mean(0), p=2, dim=-1)
        out[k] = float(torch.norm(z - cents[label_dict[c]], p=2).item())
    return out


def run_eval(real_dir, real_kp_dir, gen_dir, gen_kp_dir, state_dict, dims_raw, dims_diff, workers=0,
             timings: Optional[dict] = None, hp: Optional[dict] = None):
    """Full eval.py flow; returns (combined_scores, extras).  hp: the checkpoint's d_model / time_layers /
    time_heads (load_model, eval.py:136-152; default 256 / 4 / 8)."""
    t0 = time.perf_counter()
    real = scan_real(real_dir)
    train = split(real)
    stats = compute_stats(train, real_kp_dir)
    t1 = time.perf_counter()
    enc = OracleEncoder(state_dict, dims_raw, dims_diff, **(hp or {}))
    label_dict = {c: i for i, c in enumerate(sorted(real.keys()))}
    cents, counts = centroids(enc, train, real_kp_dir, stats, label_dict)
    t2 = time.perf_counter()
    items = scan_generated(gen_dir)
    samples = [(cls, name, path, s) for cls, name, path, T in items for s in windows_for(T)]
    seq, fe, clss, names = encode_samples(enc, samples, gen_kp_dir, stats, batch_size=32, workers=workers)
    t3 = time.perf_counter()
    ac = ac_scores(seq, clss, names, cents, label_dict)
    tc = tc_scores(fe, names)
    t4 = time.perf_counter()
    combined = {}
    for v in sorted(set(ac) | set(tc)):
        e = {}
        if v in ac:
            e["ac"] = ac[v]
        if v in tc:
            e["tc"] = tc[v]
        combined[v] = e
    if timings is not None:
        timings.update(stats_s=t1 - t0, centroids_s=t2 - t1, gen_extract_s=t3 - t2, metrics_s=t4 - t3,
                       n_videos=len(items), n_windows=len(samples))
    return combined, {"stats": stats, "centroids": cents, "counts": counts, "label_dict": label_dict,
                      "seq": seq, "frame_embeds": fe, "train": train}
