"""Multi-GPU (one process per GPU) composition of the scoring path -- SURVEY.md section 8(e).

The path shards: videos and windows are independent.  Each rank
  * takes a contiguous block of the sorted real-train video list and of the sorted generated video list,
  * accumulates its ModalityStats sufficient statistics (float64 column sums + frame counts) and its
    real-class centroid sufficient statistics (float32 sums [C,256] + counts [C]) on its GPU,
  * exchanges those (~52 KB) with ONE all-gather each and sums the gathered partials in rank order, so every
    rank finalises bit-identical stats / centroids whatever the collective's reduction order,
  * scores its generated videos (no collective in the scoring step) and the per-video (ac, tc) dicts are
    gathered to rank 0, which writes video_scores.json.
Backends: "nccl" (= RCCL over xGMI) for the production launch (bench.py / torchrun); "gloo" works on CPU
tensors and is what the world_size-2 CPU tests use.  Nothing here is specific to a rank count.
"""
from __future__ import annotations

import json
import os
import time
from concurrent.futures import Future, ThreadPoolExecutor
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist


def world() -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_bounds(n: int, rank: int, world_size: int) -> Tuple[int, int]:
    """Contiguous block [lo, hi) of n items for `rank`; the first n % world ranks take one extra item."""
    q, r = divmod(n, world_size)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def shard(items: Sequence, rank: int, world_size: int) -> List:
    lo, hi = shard_bounds(len(items), rank, world_size)
    return list(items[lo:hi])


def _collective_device(t: torch.Tensor) -> torch.device:
    # gloo collectives run on host tensors; nccl (RCCL) on device tensors
    return torch.device("cpu") if dist.get_backend() == "gloo" else t.device


def allgather_sum(t: torch.Tensor) -> torch.Tensor:
    """All-gather `t` from every rank and sum the parts in rank order (deterministic, identical on all
    ranks).  Returns a tensor on t's device and dtype."""
    rank, ws = world()
    if ws == 1:
        return t
    src = t.detach().to(_collective_device(t)).contiguous()
    parts = [torch.empty_like(src) for _ in range(ws)]
    dist.all_gather(parts, src)
    out = parts[0].clone()
    for p in parts[1:]:
        out += p
    return out.to(t.device)


def stats_reduce_fn(sums: torch.Tensor, counts: np.ndarray):
    """reduce_fn for vge.eval.compute_stats_from_npz: float64 sums [2,2596] + int64 frame counts [2]."""
    s = allgather_sum(sums)
    c = allgather_sum(torch.as_tensor(np.asarray(counts, np.int64)))
    return s, c.cpu().numpy().astype(np.int64)


def centroid_reduce_fn(sums: torch.Tensor, counts: torch.Tensor):
    """reduce_fn for vge.eval.build_real_centroids: float32 sums [C,256] + counts [C]."""
    return allgather_sum(sums), allgather_sum(counts)


def gather_to_rank0(obj):
    """Gather a picklable per-rank result (here: the per-video score dicts) to rank 0 (list in rank
    order); other ranks get None."""
    rank, ws = world()
    if ws == 1:
        return [obj]
    out = [None] * ws if rank == 0 else None
    dist.gather_object(obj, out, dst=0)
    return out


def merge_scores(parts: List[Dict[str, dict]]) -> Dict[str, dict]:
    merged = {}
    for p in parts:
        for k, v in p.items():
            if k in merged:
                raise ValueError(f"video {k} scored on two ranks")
            merged[k] = v
    return dict(sorted(merged.items()))


def run_eval_distributed(generated_meshes_dir: str, real_meshes_dir: str, model_path, keypoint_dir: str,
                         real_kp_dir: str, clip_len: int = 32, stride: int = 8,
                         out_json: Optional[str] = "video_scores.json", device="cuda", compute: str = "f32x3",
                         timings: Optional[dict] = None):
    """vge.eval.run_eval sharded over the ranks of the initialised process group.  Returns the merged
    {video: {ac, tc}} dict on rank 0 (None elsewhere); rank 0 writes out_json."""
    from . import eval as VE
    from .data import NpzVideoDataset, create_dataset_from_generated_meshes
    rank, ws = world()
    t0 = time.perf_counter()
    # The generated set's npz decode (host threads, GIL released) runs in the background while the real set's
    # statistics, the checkpoint load and the centroids proceed; its errors surface where the reference's
    # generated-set pass would raise them (after the centroids).
    gen = create_dataset_from_generated_meshes(generated_meshes_dir)
    gen_items = sorted(gen.items, key=lambda it: it.path)
    mine = NpzVideoDataset("", items=shard(gen_items, rank, ws))
    overlap = os.environ.get("VGE_FLOW_OVERLAP", "1") != "0"  # 0: every phase in order (A/B timing)
    pool = ThreadPoolExecutor(max_workers=2)
    gen_fs = pool.submit(VE.load_frame_store, mine.items, keypoint_dir, True) if mine.items and overlap else None
    if overlap and isinstance(model_path, (str, os.PathLike)):  # the checkpoint read overlaps the real set's phases
        model_path = pool.submit(VE._load_state_dict, model_path)
    try:
        return _run_eval_phases(generated_meshes_dir, real_meshes_dir, model_path, keypoint_dir, real_kp_dir,
                                clip_len, stride, out_json, device, compute, timings, rank, ws, t0, mine, gen_fs)
    finally:
        pool.shutdown(wait=True)


def _run_eval_phases(generated_meshes_dir, real_meshes_dir, model_path, keypoint_dir, real_kp_dir, clip_len, stride,
                     out_json, device, compute, timings, rank, ws, t0, mine, gen_fs):
    from . import eval as VE
    from . import ops
    from .data import ACTION_CLASSES, NpzVideoDataset, load_clip, train_test_split
    real_ds = NpzVideoDataset(real_meshes_dir, filter_classes=ACTION_CLASSES)
    train_ds, _ = train_test_split(real_ds, train_ratio=0.8, seed=1337)
    my_train = shard(train_ds.items, rank, ws)
    label_dict = {cls: i for i, cls in enumerate(sorted({it.cls for it in real_ds.items}))}
    real_store = None
    if my_train:
        real_store = ops.DeviceFrameStore.from_host(VE.load_frame_store(my_train, real_kp_dir, False), device)
        stats = VE.compute_stats_from_npz(my_train, real_kp_dir, device=device, store=real_store,
                                          reduce_fn=stats_reduce_fn)
    else:  # an empty shard still takes part in the collectives
        sums = torch.zeros((2, ops.FEAT_DIM), device=device, dtype=torch.float64)
        s, c = stats_reduce_fn(sums, np.zeros(2, np.int64))
        mean, std = ops.stats_finalize(s, c)
        stats = VE.ModalityStatsGPU(mean, std, s, c)
    dims_raw, dims_diff = VE.infer_dims_from_stats(stats)
    if isinstance(model_path, Future):
        model_path = model_path.result()  # (state_dict, hyper-parameters); a read error surfaces here, as before
    model = VE.load_model(model_path, dims_raw, dims_diff, device=device, compute=compute)
    t1 = time.perf_counter()
    if real_store is not None:
        for i, it in enumerate(my_train):
            if real_store.host_videos[i, 3] == 0:
                load_clip(it, real_kp_dir, require_kp=True)  # raises like utils.py:416-417
    centroids, label_dict, _ = VE.build_real_centroids(model, real_meshes_dir, real_kp_dir, stats, clip_len, stride,
                                                       device, train_items=my_train, label_dict=label_dict,
                                                       store=real_store, reduce_fn=centroid_reduce_fn)
    t2 = time.perf_counter()
    combined = {}
    if mine.items:
        fs = gen_fs.result() if gen_fs is not None else VE.load_frame_store(mine.items, keypoint_dir, True)
        store = ops.DeviceFrameStore.from_host(fs, device)
        feats = VE.extract_window_features(model, mine, keypoint_dir, stats, clip_len, stride, device, store=store)
        ac = VE.compute_action_consistency_scores(feats, centroids, label_dict)
        tc = VE.compute_temporal_coherence_scores(feats, centroids, label_dict)
        combined = VE.combine_scores(ac, tc)
    if torch.cuda.is_available() and str(device).startswith("cuda"):
        torch.cuda.synchronize(device)
    t3 = time.perf_counter()
    parts = gather_to_rank0(combined)
    if timings is not None:
        timings.update(stats_s=t1 - t0, centroids_s=t2 - t1, gen_s=t3 - t2, rank=rank, world=ws)
    if rank != 0:
        return None
    merged = merge_scores(parts)
    if out_json:
        with open(out_json, "w") as f:
            json.dump(merged, f, indent=2)
    return merged
