"""Extraction drivers around the GPU extractors: the callers and on-disk formats either side of them.

Mirrors the reference's extraction scripts, minus video decoding (cv2 is not part of this framework: callers pass
decoded uint8 RGB frames):

  extract_mesh.py:12-43       mesh_info_to_arrays / save_video_npz -- one np.savez_compressed per video with
                              pose / betas / global_orient / vit / frame_idx / meta (JSON string); the file the scorer's
                              npz reader (vge.ingest, utils.py:383-424) consumes
  mesh_generator.py:101-117   the single-person gate: a frame is used only with exactly one person box; a video with
                              fewer than 80 % such frames is rejected (process_video returns False)
  extract_mesh.py:157-246     per video: process_video -> save_video_npz under <out_root>/<action>/<stem>.npz, or the
                              video goes to the not-single list
  process_video.py:59-91      per video: keypoints.npy [T', 120] float32 under <root>/<action>/<stem>/

The per-frame models run on the GPU (vge.hmr.HmrExtractor, vge.dwpose.Wholebody); nothing here computes features.
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import Dict, Optional, Sequence, Union

import numpy as np

SINGLE_PERSON_MIN_FRACTION = 0.8   # mesh_generator.py:116 (len(valid_frames) < 0.8 * len(frames) -> False)


def mesh_info_to_arrays(mesh_info: dict):
    """extract_mesh.py:12-23: {frame_idx: {pose, betas, global_orient, vit}} -> float32 arrays in frame order."""
    frame_ids = sorted(mesh_info.keys())
    pose = np.stack([mesh_info[i]["pose"] for i in frame_ids]).astype(np.float32)
    betas = np.stack([mesh_info[i]["betas"] for i in frame_ids]).astype(np.float32)
    gori = np.stack([mesh_info[i]["global_orient"] for i in frame_ids]).astype(np.float32)
    vit = np.stack([mesh_info[i]["vit"] for i in frame_ids]).astype(np.float32)
    return pose, betas, gori, vit, np.asarray(frame_ids, dtype=np.int32)


def save_video_npz(video_id: str, mesh_info: dict, out_root: Union[str, Path] = "meshes_npz",
                   meta: Optional[dict] = None) -> str:
    """extract_mesh.py:25-43: <out_root>/<dirname(video_id)>/<basename(video_id)>.npz, np.savez_compressed."""
    pose, betas, gori, vit, frames = mesh_info_to_arrays(mesh_info)
    out_dir = Path(out_root) / Path(video_id).parent
    out_dir.mkdir(parents=True, exist_ok=True)
    out_path = out_dir / f"{Path(video_id).name}.npz"
    np.savez_compressed(out_path, pose=pose, betas=betas, global_orient=gori, vit=vit, frame_idx=frames,
                        meta=json.dumps(meta or {}, ensure_ascii=False))
    return str(out_path)


def single_person_frames(person_counts: Sequence[int]) -> Optional[np.ndarray]:
    """mesh_generator.py:101-117: indices of the frames with exactly one person box, or None when there are none
    or fewer than 80 % of the frames qualify (the reference's `return False`)."""
    counts = np.asarray(person_counts)
    valid = np.flatnonzero(counts == 1)
    if valid.size == 0 or valid.size < SINGLE_PERSON_MIN_FRACTION * counts.size:
        return None
    return valid


def process_video(hmr, crops, person_counts: Optional[Sequence[int]] = None):
    """MeshGenerator.process_video: TokenHMR on the single-person frames' crops -> mesh_info {frame_idx: {...}}, or
    False for a rejected video.  crops: uint8 [F, 256, 256, 3] RGB person crops on the device (one per frame; the
    box crop / ViTDetDataset warp is upstream), person_counts: detector boxes per frame (None = every frame has
    exactly one person)."""
    import torch
    F = int(crops.shape[0])
    idx = np.arange(F) if person_counts is None else single_person_frames(person_counts)
    if idx is None or F == 0:
        return False
    sel = crops if idx.size == F else crops[torch.as_tensor(idx, device=crops.device)]
    out = {k: v.cpu().numpy() for k, v in hmr.extract(sel).items()}
    return {int(f): {"pose": out["pose"][j].reshape(23, 3, 3), "betas": out["betas"][j],
                     "global_orient": out["global_orient"][j].reshape(1, 3, 3), "vit": out["vit"][j]}
            for j, f in enumerate(idx)}


def keypoint_rows(wholebody, frames) -> np.ndarray:
    """process_video.py:71-84 for one video: DWposeDetector + flatten_first_person_no_padding on every frame ->
    float32 [T', 120] (with the whole-frame fallback every frame yields a row)."""
    return np.asarray(wholebody(frames).cpu().numpy(), dtype=np.float32)


def save_keypoints(rows: np.ndarray, root: Union[str, Path], action: str, vid_id: str) -> str:
    """process_video.py:68, 83-85: <root>/<action>/<vid_id>/keypoints.npy."""
    out = Path(root) / action / vid_id / "keypoints.npy"
    out.parent.mkdir(parents=True, exist_ok=True)
    np.save(out, np.asarray(rows, dtype=np.float32))
    return str(out)


def extract_video(hmr, wholebody, frames, crops, action: str, video: str, mesh_root, kp_root,
                  person_counts: Optional[Sequence[int]] = None, source_path: str = "") -> Dict[str, Optional[str]]:
    """One video of extract_mesh.py:main + process_video.py: npz (or None when the single-person gate rejects the
    video, the reference's not-single list) and keypoints.npy paths."""
    stem = Path(video).stem
    mesh_info = process_video(hmr, crops, person_counts)
    npz = None
    if mesh_info:
        npz = save_video_npz(str(Path(action) / stem), mesh_info, out_root=mesh_root,
                             meta={"action": action, "video": video, "source_path": source_path})
    kp = save_keypoints(keypoint_rows(wholebody, frames), kp_root, action, stem)
    return {"npz": npz, "keypoints": kp}
