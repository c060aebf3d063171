"""On-disk feature ingest on libvge's native decoder (include/vge_ingest.h).

The reference reads every video with np.load (utils.py:383-424: the npz of extract_mesh.py:35-43 and the
keypoints.npy), in DataLoader worker processes.  Here one call decodes a whole list of videos with a pool
of native threads: the zip central directory is parsed and each member raw-deflate inflated straight into
the frame-store arrays (vge.data.FrameStore), allocated in pinned host memory when a GPU is present so the
upload to HBM is a plain DMA.

    load_frame_store_native(items, keypoint_dir, require_kp)   -> FrameStore   (same contents as
                                                                   eval.load_frame_store's numpy reader)
    save_sidecar(store, path) / load_sidecar(path)             -> a packed, uncompressed frame-store file:
                                                                   repeated evaluations skip zlib entirely

Error behaviour follows vge.data.load_clip: a missing keypoints.npy raises FileNotFoundError when
require_kp (utils.py:416-417) and leaves the video without keypoints otherwise (utils.py:669-678); an
unreadable keypoints.npy raises RuntimeError when require_kp; an unreadable npz raises RuntimeError.
"""
from __future__ import annotations

import ctypes as C
import json
import os
from typing import Optional, Sequence

import numpy as np
import torch

from . import lib as L
from .data import FrameStore, VideoItem, keypoint_path

SIDECAR_MAGIC = b"VGEFS001"


def _alloc(shape, pinned: bool) -> np.ndarray:
    if pinned:
        return torch.empty(shape, dtype=torch.float32, pin_memory=True).numpy()
    return np.empty(shape, np.float32)


def _cstrs(strs):
    arr = (C.c_char_p * len(strs))()
    arr[:] = [None if s is None else s.encode() for s in strs]
    return arr


def load_frame_store_native(items: Sequence[VideoItem], keypoint_dir: Optional[str], require_kp: bool,
                            threads: int = 0, pinned: Optional[bool] = None) -> FrameStore:
    lib = L.load()
    n = len(items)
    if pinned is None:
        pinned = torch.cuda.is_available()
    npz = [it.path for it in items]
    kps = [None] * n
    if keypoint_dir is not None:
        for i, it in enumerate(items):
            kps[i] = keypoint_path(keypoint_dir, it.cls, os.path.splitext(os.path.basename(it.path))[0])
    c_npz, c_kp = _cstrs(npz), _cstrs(kps)
    info = (L.ClipInfo * max(n, 1))()
    lib.vge_ingest_probe(c_npz, c_kp, n, threads, info)
    lens, klens = [], []
    for i in range(n):
        st, kf = info[i].status, info[i].kp_frames
        if st in (1, 7, 8):
            raise RuntimeError(f"vge_ingest: cannot read '{npz[i]}' ({L.INGEST_STATUS.get(st, st)})")
        if st == 9:  # keypoints.npy present but unreadable
            if require_kp:
                raise RuntimeError(f"Failed to load keypoints from '{kps[i]}' for video "
                                   f"'{os.path.splitext(os.path.basename(npz[i]))[0]}'")
            kf, kps[i] = -1, None
        if kf < 0 and keypoint_dir is not None and require_kp:
            stem = os.path.splitext(os.path.basename(npz[i]))[0]
            raise FileNotFoundError(f"Expected keypoints at '{kps[i]}' for video '{stem}' but file does not exist.")
        lens.append(int(info[i].n_frames))
        klens.append(max(int(kf), 0))
    vit_dim = int(info[0].vit_dim) if n else 1024
    if any(int(info[i].vit_dim) != vit_dim for i in range(n)):
        raise RuntimeError("vge_ingest: videos with different vit dims cannot share one frame store")
    F, Fk = sum(lens), sum(klens)
    store = FrameStore(pose=_alloc((F, 207), pinned), gori=_alloc((F, 9), pinned), betas=_alloc((F, 10), pinned),
                       vit=_alloc((F, vit_dim), pinned), kp=_alloc((max(Fk, 1), 120), pinned),
                       videos=np.zeros((n, 4), np.int32), names=[it.name for it in items],
                       classes=[it.cls for it in items])
    off = koff = 0
    for i in range(n):
        store.videos[i] = (off, lens[i], koff, klens[i])
        off += lens[i]
        koff += klens[i]
    status = np.zeros(max(n, 1), np.int32)
    c_kp = _cstrs(kps)
    ptr = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    rc = lib.vge_ingest_decode(c_npz, c_kp, n, threads, ptr(store.videos), vit_dim, ptr(store.pose),
                               ptr(store.gori), ptr(store.betas), ptr(store.vit), ptr(store.kp), ptr(status))
    if rc != 0:
        bad = int(np.flatnonzero(status[:n])[0])
        raise RuntimeError(f"vge_ingest: decoding '{npz[bad]}' failed ({L.INGEST_STATUS.get(int(status[bad]))})")
    return store


# ----------------------------------------------------------------------------- packed sidecar

_ARRAYS = ("pose", "gori", "betas", "vit", "kp", "videos")


def _layout(meta: dict, data_start: int):
    offs, pos = {}, data_start
    for k in _ARRAYS:
        spec = meta["arrays"][k]
        pos = (pos + 4095) // 4096 * 4096
        offs[k] = pos
        pos += int(np.prod(spec["shape"])) * np.dtype(spec["dtype"]).itemsize
    return offs


def save_sidecar(store: FrameStore, path: str) -> None:
    """One uncompressed file: magic, u64 header length, JSON header (names, classes, shapes), then the
    arrays in _ARRAYS order, each starting on a 4 KiB boundary."""
    arrays = {k: np.ascontiguousarray(getattr(store, k)) for k in _ARRAYS}
    meta = {"names": list(store.names), "classes": list(store.classes),
            "arrays": {k: {"shape": list(a.shape), "dtype": a.dtype.str} for k, a in arrays.items()}}
    head = json.dumps(meta).encode()
    offs = _layout(meta, len(SIDECAR_MAGIC) + 8 + len(head))
    with open(path, "wb") as f:
        f.write(SIDECAR_MAGIC)
        f.write(np.uint64(len(head)).tobytes())
        f.write(head)
        for k in _ARRAYS:
            f.seek(offs[k])
            f.write(arrays[k].tobytes())


def load_sidecar(path: str, pinned: Optional[bool] = None) -> FrameStore:
    if pinned is None:
        pinned = torch.cuda.is_available()
    with open(path, "rb") as f:
        if f.read(len(SIDECAR_MAGIC)) != SIDECAR_MAGIC:
            raise RuntimeError(f"'{path}' is not a vge frame-store sidecar")
        hl = int(np.frombuffer(f.read(8), np.uint64)[0])
        meta = json.loads(f.read(hl))
        offs = _layout(meta, len(SIDECAR_MAGIC) + 8 + hl)
        out = {}
        for k in _ARRAYS:
            spec = meta["arrays"][k]
            a = (_alloc(tuple(spec["shape"]), pinned) if spec["dtype"] == "<f4"
                 else np.empty(tuple(spec["shape"]), np.dtype(spec["dtype"])))
            f.seek(offs[k])
            if f.readinto(memoryview(a).cast("B")) != a.nbytes:
                raise RuntimeError(f"'{path}': truncated array {k}")
            out[k] = a
    return FrameStore(names=meta["names"], classes=meta["classes"], **out)
