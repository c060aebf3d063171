"""The deterministic synthetic dataset behind the golden fixtures (shared by make_golden.py and the
tests, so both sides see byte-identical inputs; `digest` guards against generator drift)."""
from __future__ import annotations

import hashlib
import os
from pathlib import Path

import numpy as np

from vge import synth

GOLDEN_SPEC = {
    "n_real_per_class": 4,
    "T_real": (32, 40, 64, 20),
    "n_gen": 16,
    "T_gen": (32, 64, 20, 45, 33),
    "kp_short_every": 3,
    "feat_windows": [0, 5, 13],
}


NOKP_MODS = ("vit", "global", "pose", "beta")  # the keypoint-less model (keypoint_dir None, utils.py:496-514)
# a checkpoint of another shape (load_model reads d_model / time_layers / time_heads from it, eval.py:136-152)
SMALL_HP = {"d_model": 64, "time_layers": 2, "time_heads": 4}


def golden_state_dict(layout: str = "kp"):
    """The golden checkpoint's weights: 5 modalities, or the keypoint-less 4 (same generator, no kp2d), or "small":
    5 modalities at SMALL_HP's shape."""
    if layout == "small":
        return synth.make_state_dict(synth.DIMS_RAW, synth.DIMS_DIFF, d_model=SMALL_HP["d_model"],
                                     time_layers=SMALL_HP["time_layers"])
    if layout == "kp":
        return synth.make_state_dict(synth.DIMS_RAW, synth.DIMS_DIFF)
    return synth.make_state_dict({m: synth.DIMS_RAW[m] for m in NOKP_MODS},
                                 {m: synth.DIMS_DIFF[m] for m in NOKP_MODS})


def build_golden_dataset(root: str, layout: str = "kp"):
    """Write dataset + checkpoint under `root`; returns (paths, checkpoint_path, sha256 hexdigest).  layout "nokp":
    the same dataset with the 4-modality checkpoint (model_nokp.pt) of the keypoint-less flow; "small": the
    5-modality flow with a d_model 64, 2-layer, 4-head checkpoint (model_small.pt)."""
    paths = synth.write_dataset(root, n_real_per_class=GOLDEN_SPEC["n_real_per_class"],
                                n_gen=GOLDEN_SPEC["n_gen"], T_real=GOLDEN_SPEC["T_real"],
                                T_gen=GOLDEN_SPEC["T_gen"], kp_short_every=GOLDEN_SPEC["kp_short_every"])
    # one generated clip whose filename carries no known action -> class "Testmodel", no AC score
    clip = synth.make_clip(synth.SEED_GEN, 999, 32)
    stem = "Testmodel_Xyzzy_00_deadbeef"
    synth.save_clip_npz(Path(paths["generated_meshes"]) / f"{stem}.npz", clip)
    kd = Path(paths["generated_kps"]) / stem
    kd.mkdir(parents=True, exist_ok=True)
    np.save(kd / "keypoints.npy", clip.keypoints)
    sd = golden_state_dict(layout)
    ckpt = os.path.join(root, {"kp": "model.pt", "nokp": "model_nokp.pt", "small": "model_small.pt"}[layout])
    synth.save_checkpoint(ckpt, sd, **(SMALL_HP if layout == "small" else {}))
    h = hashlib.sha256()
    for sub in ("real", "real_kp", "generated_meshes", "generated_kps"):
        for p in sorted(Path(paths[sub]).rglob("*")):
            if p.suffix == ".npz":
                with np.load(p) as z:
                    for k in ("pose", "global_orient", "betas", "vit"):
                        h.update(np.ascontiguousarray(z[k]).tobytes())
            elif p.suffix == ".npy":
                h.update(np.load(p).tobytes())
    for k in sorted(sd):
        h.update(k.encode())
        h.update(np.ascontiguousarray(sd[k]).tobytes())
    return paths, ckpt, h.hexdigest()
