"""Extraction drivers around the GPU extractors: the callers and on-disk formats either side of them.

Mirrors the reference's extraction scripts, minus video decoding (cv2 is not part of this framework: callers pass
decoded uint8 RGB frames):

  mesh_generator.py:101-145   the TokenHMR front end: person detection (detectron2 Faster R-CNN X101-32x8d-FPN,
                              vge.frcnn), the single-person gate (exactly one person instance with score > 0.5 per
                              frame, >= 80 % of the frames), ViTDetDataset's crop (vge_hmr_crop)

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
PERSON_SCORE_THRESH = 0.5          # mesh_generator.py:107 (pred_classes == 0) & (scores > 0.5): vge_frcnn's gate_thresh


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


def gate_videos(keep: np.ndarray, frames_per_video: int, frame_off: int = 0):
    """mesh_generator.py:101-117 over a batch of equal-length videos laid out back to back: keep [n_videos * T] per-frame
    single-person flags -> (accepted video indices, kept frame indices into the batch, descriptor rows
    {frame_off, n_frames, kp_off, kp_frames} of the accepted videos' frame-store entries: the npz holds the kept frames
    only (compacted from `frame_off` on, extract_mesh.py:35-43), keypoints.npy every frame (process_video.py))."""
    keep = np.asarray(keep, bool)
    T = int(frames_per_video)
    nv = keep.size // T
    acc, kept, desc = [], [], []
    off = int(frame_off)
    for v in range(nv):
        valid = single_person_frames(np.where(keep[v * T:(v + 1) * T], 1, 0))
        if valid is None:
            continue
        acc.append(v)
        kept.append(valid + v * T)
        desc.append((off, valid.size, v * T, T))
        off += valid.size
    kept_idx = np.concatenate(kept) if kept else np.zeros(0, np.int64)
    return np.asarray(acc, np.int64), kept_idx, np.asarray(desc, np.int32).reshape(-1, 4)


def gate_mask(n_person) -> np.ndarray:
    """mesh_generator.py:103-111 per frame: exactly one (pred_classes == 0) & (scores > 0.5) instance of the gate
    detector (vge.frcnn.FrcnnDetector's n_person)."""
    return np.asarray(n_person).reshape(-1) == 1


def tokenhmr_front(detector, frames, detections=None):
    """TokenHMRMeshGenerator.process_video's front end (mesh_generator.py:101-145) on the device: detectron2's Faster
    R-CNN X101-32x8d-FPN on every frame (vge.frcnn.FrcnnDetector, the reference's det2_predictor), the per-frame
    single-person gate, the 80 % rule, and ViTDetDataset's crop of every kept frame around its one person box.
    frames: uint8 [F, H, W, 3] RGB on the device; detections: optional (person boxes [F, 4] -- the first class-0
    instance of each frame --, n_person [F]) host arrays already computed for these frames.  Returns (kept frame
    indices, uint8 crops [n, 256, 256, 3] on the device), or None when the reference rejects the video
    (process_video returns False)."""
    from .hmr import crop_persons
    if detections is None:
        out = detector.detect(frames)
        boxes, npers = out["person"][:, 0, :4].cpu().numpy(), out["n_person"].cpu().numpy()
    else:
        boxes, npers = np.asarray(detections[0], np.float32).reshape(-1, 4), np.asarray(detections[1])
    keep = np.flatnonzero(gate_mask(npers))
    F = int(frames.shape[0])
    if keep.size == 0 or keep.size < SINGLE_PERSON_MIN_FRACTION * F:
        return None
    return keep, crop_persons(frames, boxes[keep], keep)


def process_video_frames(hmr, detector, frames, detections=None):
    """TokenHMRMeshGenerator.process_video (mesh_generator.py:91-171) from full frames: front end (detector, gate,
    crops) then TokenHMR on the kept frames -> {frame_idx: {pose [23,3,3], betas, global_orient [1,3,3], vit}} or
    False."""
    front = tokenhmr_front(detector, frames, detections)
    if front is None:
        return False
    idx, crops = front
    out = {k: v.cpu().numpy() for k, v in hmr.extract(crops).items()}
    return {int(f): {"pose": out["pose"][j].reshape(23, 3, 3), "betas": out["betas"][j],
                     "global_orient": out["global_orient"][j].reshape(1, 3, 3), "vit": out["vit"][j]}
            for j, f in enumerate(idx)}


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
                  person_counts: Optional[Sequence[int]] = None, source_path: str = "",
                  detector=None) -> Dict[str, Optional[str]]:
    """One video of extract_mesh.py:main + process_video.py: npz (or None when the single-person gate rejects the
    video, the reference's not-single list) and keypoints.npy paths.  crops None: the TokenHMR front end runs on the
    full frames with `detector` (a vge.frcnn.FrcnnDetector: process_video_frames); otherwise crops are ready-made person
    crops.  DWPose (`wholebody`) runs its own YOLOX-L persons on every frame, as process_video.py does."""
    stem = Path(video).stem
    if crops is None:
        if detector is None:
            raise ValueError("extract_video: the TokenHMR front end needs the gate detector (vge.frcnn.FrcnnDetector)")
        mesh_info = process_video_frames(hmr, detector, frames)
    else:
        mesh_info = process_video(hmr, crops, person_counts)
    npz = None
    if mesh_info:
        npz = save_video_npz(str(Path(action) / stem), mesh_info, out_root=mesh_root,
                             meta={"action": action, "video": video, "source_path": source_path})
    kp = save_keypoints(keypoint_rows(wholebody, frames), kp_root, action, stem)
    return {"npz": npz, "keypoints": kp}


def extract_videos(hmr, wholebody, detector, videos, mesh_root, kp_root, max_frames: int = 1024) -> Dict[str, Optional[str]]:
    """extract_mesh.py:150-241 + process_video.py:59-94 over a list of videos, batched for the GPU: videos are
    (stem, uint8 [T, H, W, 3] device frames) of any lengths; consecutive videos are packed into passes of at most
    `max_frames` frames (a longer video is a pass of its own), and each pass runs the gate detector (detectron2 Faster
    R-CNN, `detector`) and DWPose (`wholebody`: YOLOX-L persons -> RTMPose-l) once over all its frames, then TokenHMR
    once over the crops of every kept frame of the pass's accepted videos.  Per video, as the reference does one at a
    time: the single-person gate and its 80 % rule (mesh_generator.py:101-117), <mesh_root>/<stem>.npz of the kept
    frames (extract_mesh.py:35-43; a rejected video gets none: the not-single list) and
    <kp_root>/<stem>/keypoints.npy of every frame (process_video.py writes them for every video).
    Returns {stem: npz path or None}."""
    import torch
    from .hmr import crop_persons
    out: Dict[str, Optional[str]] = {}
    passes, cur, n = [], [], 0
    for stem, fr in videos:
        t = int(fr.shape[0])
        if cur and n + t > max_frames:
            passes.append(cur)
            cur, n = [], 0
        cur.append((stem, fr))
        n += t
    if cur:
        passes.append(cur)
    for group in passes:
        fr = group[0][1] if len(group) == 1 else torch.cat([f for _, f in group], 0)
        det = detector.detect(fr)
        kp = wholebody(fr).cpu().numpy()
        boxes = det["person"][:, 0, :4].cpu().numpy()
        npers = det["n_person"].cpu().numpy()
        kept, spans, f0 = [], [], 0
        for stem, f in group:
            t = int(f.shape[0])
            valid = single_person_frames(np.where(gate_mask(npers[f0:f0 + t]), 1, 0))
            spans.append((stem, f0, t, valid))
            if valid is not None:
                kept.append(valid + f0)
            f0 += t
        rows = None
        if kept:
            kf = np.concatenate(kept)
            crops = crop_persons(fr, boxes[kf], kf)
            rows = {k: v.cpu().numpy() for k, v in hmr.extract(crops).items()}
        r = 0
        for stem, f0, t, valid in spans:
            save_keypoints(kp[f0:f0 + t], Path(kp_root), "", stem)
            if valid is None:
                out[stem] = None
                continue
            mesh_info = {int(fi): {"pose": rows["pose"][r + j].reshape(23, 3, 3), "betas": rows["betas"][r + j],
                                   "global_orient": rows["global_orient"][r + j].reshape(1, 3, 3),
                                   "vit": rows["vit"][r + j]} for j, fi in enumerate(valid)}
            r += valid.size
            out[stem] = save_video_npz(stem, mesh_info, out_root=mesh_root, meta={"video": stem})
    return out
