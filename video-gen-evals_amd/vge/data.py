"""Host-side data layer: the reference's dataset scan, split and window enumeration, plus the
packing of per-frame features into the contiguous HBM "frame store" the HIP kernels read.

Mirrors (same names, argument meaning and error behaviour):
  ACTION_CLASSES / _canonicalize_class      eval.py:22-45
  VideoItem                                 utils.py:221-227
  NpzVideoDataset (scan <root>/<Class>/*.npz, sorted; unreadable files skipped)  utils.py:229-324
  train_test_split (random.Random(seed) per class, banker's round)               utils.py:326-341
  create_dataset_from_generated_meshes (class from filename tokens)              eval.py:48-101
  sample_all_windows_npz (generated set: T<32 -> one window at 0)                utils.py:888-911
  enumerate_test_windows (make_test_loader's sample list, length<=0 skipped)      utils.py:803-844
  keypoint_path (flat dir if its name has SAVE_GEN/SAVE_NEW/generated_kps)       utils.py:410-417
    (or an explicit "flat" / "per_class" layout: set_keypoint_layout, VGE_KP_LAYOUT, --kp-layout)

Frame store layout in HBM (one float32 array per modality, videos concatenated on the frame axis):
  pose [F,207]  global_orient [F,9]  betas [F,10]  vit [F,1024]  keypoints [Fk,120]
and one int32 descriptor per video {frame_off, n_frames, kp_off, kp_frames}.  A window is
{video, start}.  Keypoint sequences have their own length (process_video.py drops frames).
"""
from __future__ import annotations

import os
import random
from dataclasses import dataclass, field
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

ACTION_CLASSES = [
    "BodyWeightSquats", "HulaHoop", "JumpingJack", "PullUps", "PushUps",
    "Shotput", "SoccerJuggling", "TennisSwing", "ThrowDiscus", "WallPushups",
]


def _canonicalize_class(name: str) -> str:
    for cls in ACTION_CLASSES:
        if name.lower() == cls.lower():
            return cls
    aliases = {"soccerjuggling": "SoccerJuggling", "tennisswing": "TennisSwing"}
    return aliases.get(name.lower(), name)


@dataclass
class VideoItem:
    cls: str
    name: str      # file name with .npz
    path: str
    length: int    # number of frames T
    vit_dim: int


class NpzVideoDataset:
    """<root>/<Class>/*.npz scan; `items` overrides the scan (utils.py:229-324)."""

    def __init__(self, root_dir: str, items: Optional[List[VideoItem]] = None,
                 filter_classes: Optional[Sequence[str]] = None, enforce_min_per_class: bool = False):
        self.root_dir = root_dir
        self.filter_classes = list(filter_classes) if filter_classes is not None else None
        raw_items = items if items is not None else self._scan()
        class_to_items: Dict[str, List[VideoItem]] = {}
        for it in raw_items:
            class_to_items.setdefault(it.cls, []).append(it)
        if self.filter_classes is not None:
            allowed = set(self.filter_classes)
            class_to_items = {c: v for c, v in class_to_items.items() if c in allowed}
        self.class_to_items = class_to_items
        self.items = [it for vids in class_to_items.values() for it in vids]
        self.classes = sorted(class_to_items.keys())

    def _scan(self) -> List[VideoItem]:
        items: List[VideoItem] = []
        root = self.root_dir
        for cls in sorted(d for d in os.listdir(root) if os.path.isdir(os.path.join(root, d))):
            if self.filter_classes and cls not in self.filter_classes:
                continue
            cls_dir = os.path.join(root, cls)
            names = [f for f in sorted(os.listdir(cls_dir)) if f.endswith(".npz")]
            shapes = _probe_shapes([os.path.join(cls_dir, f) for f in names])
            for f, shape in zip(names, shapes):
                path = os.path.join(cls_dir, f)
                try:
                    if shape is not None:
                        T, Dv = shape
                    else:
                        with np.load(path) as npz:
                            T = int(npz["pose"].shape[0])
                            Dv = int(npz["vit"].shape[1])
                    items.append(VideoItem(cls=cls, name=f, path=path, length=T, vit_dim=Dv))
                except Exception:
                    print(f"Failed for {f}")
        return items

    def __len__(self):
        return len(self.items)

    def __getitem__(self, i):
        return self.items[i]


def train_test_split(dataset: NpzVideoDataset, train_ratio: float = 0.8, seed: int = 42):
    rng = random.Random(seed)
    train_items: List[VideoItem] = []
    test_items: List[VideoItem] = []
    for cls, vids in dataset.class_to_items.items():
        v = vids[:]
        rng.shuffle(v)
        n = len(v)
        n_train = max(1, min(n - 1, int(round(n * train_ratio))))
        train_items.extend(v[:n_train])
        test_items.extend(v[n_train:])
    return (NpzVideoDataset(dataset.root_dir, items=train_items),
            NpzVideoDataset(dataset.root_dir, items=test_items))


def _probe_shapes(paths: Sequence[str]) -> List[Optional[Tuple[int, int]]]:
    """(T, vit_dim) of each npz from its npy headers (libvge's native multithreaded probe: no payload inflate),
    None where the probe cannot read a file -- the caller then takes the reference's np.load path for that file,
    so unreadable / partial files keep the reference's behaviour exactly."""
    if not paths:
        return []
    try:
        import ctypes as C
        from . import lib as L
        lib = L.load()
    except Exception:  # the scan works without libvge (np.load for every file)
        return [None] * len(paths)
    arr = (C.c_char_p * len(paths))(*[str(p).encode() for p in paths])
    kps = (C.c_char_p * len(paths))(*([None] * len(paths)))
    info = (L.ClipInfo * len(paths))()
    lib.vge_ingest_probe(arr, kps, len(paths), 0, info)
    return [(int(info[i].n_frames), int(info[i].vit_dim)) if info[i].status == 0 else None for i in range(len(paths))]


def create_dataset_from_generated_meshes(generated_meshes_dir: str) -> NpzVideoDataset:
    items = []
    files = sorted(Path(generated_meshes_dir).glob("*.npz"))
    shapes = _probe_shapes([str(f) for f in files])
    for npz_file, shape in zip(files, shapes):
        try:
            stem = npz_file.stem
            parts = stem.split("_")
            cls_name = None
            for part in parts:
                canon = _canonicalize_class(part)
                if canon in ACTION_CLASSES:
                    cls_name = canon
                    break
            if cls_name is None:
                for part in parts:
                    if part[0].isupper() and not part.isdigit() and len(part) > 3 and \
                            part.lower() not in ["videos", "npz"]:
                        cls_name = _canonicalize_class(part)
                        break
            if cls_name is None:
                cls_name = "Unknown"
            if shape is not None:
                T, Dv = shape
            else:
                with np.load(npz_file) as npz:
                    T = int(npz["pose"].shape[0]) if "pose" in npz else 0
                    if "vit" in npz:
                        vshape = npz["vit"].shape
                        Dv = int(vshape[1]) if len(vshape) > 1 else 0
                    else:
                        Dv = 0
            items.append(VideoItem(cls=cls_name, name=npz_file.name, path=str(npz_file), length=T, vit_dim=Dv))
        except Exception as e:
            print(f"Failed to load {npz_file}: {e}")
    return NpzVideoDataset(root_dir=generated_meshes_dir, items=items)


def sample_all_windows_npz(ds: NpzVideoDataset, clip_len: int = 32, stride: int = 8) -> List[Tuple[VideoItem, int]]:
    out = []
    for it in ds.items:
        if it.length < clip_len:
            out.append((it, 0))
            continue
        for s in range(0, it.length - clip_len + 1, stride):
            out.append((it, s))
    return out


def enumerate_test_windows(ds: NpzVideoDataset, clip_len: int, stride: int,
                           filter_classes: Optional[Sequence[str]] = None) -> List[Tuple[VideoItem, int]]:
    allowed = set(filter_classes) if filter_classes else None
    samples = []
    for it in ds.items:
        if allowed is not None and it.cls not in allowed:
            continue
        if it.length <= 0:
            continue
        if it.length < clip_len:
            starts = [0]
        else:
            starts = list(range(0, it.length - clip_len + 1, max(1, stride)))
        samples.extend((it, s) for s in starts)
    if not samples:
        raise ValueError("make_test_loader: no samples found. "
                         f"{'Filter matched no classes.' if allowed else 'Dataset may be empty.'}")
    return samples


# Keypoint directory layout.  "auto" is the reference's name sniffing (utils.py:410-417: a directory whose path
# contains SAVE_GEN / SAVE_NEW / generated_kps is flat, <dir>/<stem>/keypoints.npy, any other is per class,
# <dir>/<Class>/<stem>/keypoints.npy); "flat" and "per_class" state the layout explicitly, so a directory whose
# name does not follow that convention still resolves.  Set per process (all directories) or per directory by
# set_keypoint_layout (the CLI's --kp-layout / --real-kp-layout), or for all directories by VGE_KP_LAYOUT.
KP_LAYOUTS = ("auto", "flat", "per_class")
_kp_layout = os.environ.get("VGE_KP_LAYOUT", "auto")
if _kp_layout not in KP_LAYOUTS:
    raise ValueError(f"VGE_KP_LAYOUT must be one of {KP_LAYOUTS}, got {_kp_layout!r}")
_kp_layout_by_dir: Dict[str, str] = {}


def set_keypoint_layout(layout: str, keypoint_dir: Optional[str] = None) -> None:
    """Layout for one keypoint directory, or (keypoint_dir None) the default for every directory without one."""
    global _kp_layout
    if layout not in KP_LAYOUTS:
        raise ValueError(f"keypoint layout must be one of {KP_LAYOUTS}, got {layout!r}")
    if keypoint_dir is None:
        _kp_layout = layout
    else:
        _kp_layout_by_dir[os.path.normpath(keypoint_dir)] = layout


def get_keypoint_layout(keypoint_dir: Optional[str] = None) -> str:
    if keypoint_dir is not None:
        return _kp_layout_by_dir.get(os.path.normpath(keypoint_dir), _kp_layout)
    return _kp_layout


def clear_keypoint_layouts() -> None:
    """Back to VGE_KP_LAYOUT (or auto) with no per-directory layouts."""
    global _kp_layout
    _kp_layout_by_dir.clear()
    _kp_layout = os.environ.get("VGE_KP_LAYOUT", "auto")


def keypoint_path(keypoint_dir: str, cls_name: str, vid_stem: str, layout: Optional[str] = None) -> str:
    layout = get_keypoint_layout(keypoint_dir) if layout is None else layout
    if layout not in KP_LAYOUTS:
        raise ValueError(f"keypoint layout must be one of {KP_LAYOUTS}, got {layout!r}")
    if layout == "auto":
        flat = "SAVE_GEN" in keypoint_dir or "SAVE_NEW" in keypoint_dir or "generated_kps" in keypoint_dir
    else:
        flat = layout == "flat"
    if flat:
        return os.path.join(keypoint_dir, vid_stem, "keypoints.npy")
    return os.path.join(keypoint_dir, cls_name, vid_stem, "keypoints.npy")


# ----------------------------------------------------------------------------- frame store

@dataclass
class FrameStore:
    """Host image of the HBM frame store (see module docstring)."""
    pose: np.ndarray        # [F,207] f32
    gori: np.ndarray        # [F,9]
    betas: np.ndarray       # [F,10]
    vit: np.ndarray         # [F,1024]
    kp: np.ndarray          # [Fk,120]
    videos: np.ndarray      # [V,4] int32 {frame_off, n_frames, kp_off, kp_frames}
    names: List[str] = field(default_factory=list)
    classes: List[str] = field(default_factory=list)

    @property
    def n_videos(self) -> int:
        return int(self.videos.shape[0])


def pack_frame_store(clips: Sequence[dict], names: Sequence[str], classes: Sequence[str]) -> FrameStore:
    """clips: dicts with pose [T,23,3,3], global_orient [T,1,3,3], betas [T,10], vit [T,1024],
    keypoints [T',120] or None (no keypoint file -> kp_frames = 0)."""
    V = len(clips)
    lens = [int(c["pose"].shape[0]) for c in clips]
    klens = [0 if c.get("keypoints") is None else int(c["keypoints"].shape[0]) for c in clips]
    F, Fk = sum(lens), sum(klens)
    vit_dim = int(clips[0]["vit"].shape[1]) if V else 1024
    st = FrameStore(pose=np.empty((F, 207), np.float32), gori=np.empty((F, 9), np.float32),
                    betas=np.empty((F, 10), np.float32), vit=np.empty((F, vit_dim), np.float32),
                    kp=np.empty((max(Fk, 1), 120), np.float32), videos=np.zeros((V, 4), np.int32),
                    names=list(names), classes=list(classes))
    off = koff = 0
    for i, c in enumerate(clips):
        T = lens[i]
        st.pose[off:off + T] = np.asarray(c["pose"], np.float32).reshape(T, 207)
        st.gori[off:off + T] = np.asarray(c["global_orient"], np.float32).reshape(T, 9)
        st.betas[off:off + T] = np.asarray(c["betas"], np.float32)
        st.vit[off:off + T] = np.asarray(c["vit"], np.float32)
        if klens[i]:
            st.kp[koff:koff + klens[i]] = np.asarray(c["keypoints"], np.float32)
        st.videos[i] = (off, T, koff, klens[i])
        off += T
        koff += klens[i]
    return st


def load_clip(item: VideoItem, keypoint_dir: Optional[str], require_kp: bool) -> dict:
    """npz + keypoints.npy for one video.  require_kp mirrors WindowDataset (missing kp raises,
    utils.py:416-417); stats mode tolerates a missing file (utils.py:669-678)."""
    with np.load(item.path) as npz:
        clip = {k: np.asarray(npz[k], np.float32) for k in ("pose", "global_orient", "betas", "vit")}
    clip["keypoints"] = None
    if keypoint_dir is not None:
        stem = os.path.splitext(os.path.basename(item.path))[0]
        kp_path = keypoint_path(keypoint_dir, item.cls, stem)
        if not os.path.exists(kp_path):
            if require_kp:
                raise FileNotFoundError(
                    f"Expected keypoints at '{kp_path}' for video '{stem}' but file does not exist.")
        else:
            try:
                clip["keypoints"] = np.asarray(np.load(kp_path), np.float32)
            except Exception as e:
                if require_kp:
                    raise RuntimeError(f"Failed to load keypoints from '{kp_path}' for video '{stem}': {e}")
    return clip
