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
import warnings
from concurrent.futures import Future, ThreadPoolExecutor
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist


def in_group() -> bool:
    return dist.is_available() and dist.is_initialized()


def world() -> Tuple[int, int]:
    if in_group():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _rank_device() -> torch.device:
    return torch.device("cuda", torch.cuda.current_device())


def shard_bounds(n: int, rank: int, world_size: int) -> Tuple[int, int]:
    """Contiguous block [lo, hi) of n items for `rank`; the first n % world ranks take one extra item."""
    q, r = divmod(n, world_size)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def shard(items: Sequence, rank: int, world_size: int) -> List:
    lo, hi = shard_bounds(len(items), rank, world_size)
    return list(items[lo:hi])


def _collective_device(t: torch.Tensor) -> torch.device:
    """gloo collectives run on host tensors; an nccl (RCCL) process group serves cuda tensors only, so a host
    tensor (e.g. the int64 frame counts of the stats exchange) is staged on this rank's current GPU."""
    if dist.get_backend() == "gloo":
        return torch.device("cpu")
    if t.device.type == "cuda":
        return t.device
    return _rank_device()


def allgather_sum(t: torch.Tensor) -> torch.Tensor:
    """All-gather `t` from every rank and sum the parts in rank order (deterministic, identical on all
    ranks).  Returns a tensor on t's device and dtype.  Inside a process group the collective runs even for
    one rank, so a one-GPU run exercises the same RCCL calls as eight."""
    if not in_group():
        return t
    rank, ws = world()
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


class PeerRankFailed(RuntimeError):
    """Raised on every rank whose own phase succeeded when another rank's failed (so no rank is left waiting
    in a collective the failed rank will never reach)."""


def agree(err: Optional[BaseException], phase: str) -> None:
    """One all-gather of a status flag per rank before each exchange of the flow.  The reference is a single
    process that raises at the first bad file (utils.py:416-417, eval.py:93-95); sharded, only the rank that
    owns that file sees it, so every rank learns of it here and raises together: the failing rank re-raises
    its own exception, the others PeerRankFailed naming the failed ranks."""
    rank, ws = world()
    if in_group():
        flag = torch.tensor([0 if err is None else 1], dtype=torch.int32)
        flag = flag.to(_collective_device(flag))
        parts = [torch.empty_like(flag) for _ in range(ws)]
        dist.all_gather(parts, flag)
        failed = [r for r, p in enumerate(parts) if int(p.item()) != 0]
    else:
        failed = [] if err is None else [0]
    if err is not None:
        raise err
    if failed:
        raise PeerRankFailed(f"{phase}: rank(s) {failed} failed; rank {rank} stops with them")


def guarded(phase: str, fn, *args, **kw):
    """Run one rank-local phase of the flow, then agree() with the other ranks before the next exchange."""
    err, out = None, None
    try:
        out = fn(*args, **kw)
    except Exception as e:  # re-raised by agree() on this rank, after the peers were told
        err = e
    agree(err, phase)
    return out


def gather_to_rank0(obj):
    """Gather a picklable per-rank result (here: the per-video score dicts) to rank 0 (list in rank
    order); other ranks get None."""
    rank, ws = world()
    if not in_group():
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
                         timings: Optional[dict] = None, human_scores_path: Optional[str] = None,
                         save_features: Optional[str] = None, stats_cache: Optional[str] = None):
    """vge.eval.run_eval sharded over the ranks of the initialised process group.  Returns the merged
    {video: {ac, tc}} dict on rank 0 (None elsewhere); rank 0 writes out_json, the Spearman correlations
    against `human_scores_path` (eval.py:456-464) and, with `save_features`, window_features.pt
    (eval.py:424, windows of all ranks in the single-process order: the shards are contiguous blocks of the
    sorted generated list).  stats_cache: the real set's stats + centroid artifact (vge/stats_cache.py); when every
    rank reads a matching one the real set is skipped: no stats or centroid exchange, only int32 flag gathers (the
    cache-hit agreement and agree()'s error flags) before the score gather; otherwise the full flow runs and rank 0
    writes the artifact after the exchanges."""
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
    model_sha = None
    if stats_cache:
        # the checkpoint digest runs before the first collective (the cache-hit agreement): an unreadable checkpoint on
        # one rank must stop every rank, not leave the others in the all-gather
        from .stats_cache import model_digest
        model_sha = guarded("stats cache fingerprint", model_digest, model_path)
    pool = ThreadPoolExecutor(max_workers=2)
    need_kp = keypoint_dir is not None
    gen_fs = pool.submit(VE.load_frame_store, mine.items, keypoint_dir, need_kp) if mine.items and overlap else None
    if overlap and isinstance(model_path, (str, os.PathLike)):  # the checkpoint read overlaps the real set's phases
        model_path = pool.submit(VE._load_state_dict, model_path)
    try:
        return _run_eval_phases(real_meshes_dir, model_path, keypoint_dir, real_kp_dir, clip_len, stride, out_json,
                                device, compute, timings, rank, ws, t0, mine, gen_fs, human_scores_path,
                                save_features, stats_cache, model_sha)
    finally:
        pool.shutdown(wait=True)


def all_agree(flag: bool) -> bool:
    """True iff `flag` holds on every rank (one int32 all-gather)."""
    if not in_group():
        return flag
    _, ws = world()
    t = torch.tensor([1 if flag else 0], dtype=torch.int32)
    t = t.to(_collective_device(t))
    parts = [torch.empty_like(t) for _ in range(ws)]
    dist.all_gather(parts, t)
    return all(int(p.item()) == 1 for p in parts)


def _run_eval_phases(real_meshes_dir, model_path, keypoint_dir, real_kp_dir, clip_len, stride, out_json, device,
                     compute, timings, rank, ws, t0, mine, gen_fs, human_scores_path, save_features, stats_cache=None,
                     model_sha=None):
    """Three rank-local phases, each closed by agree() before its exchange, so an error on one rank (a missing
    keypoints.npy, an unreadable checkpoint) makes every rank raise instead of leaving peers in a collective."""
    from . import eval as VE
    from . import ops
    from .data import ACTION_CLASSES, NpzVideoDataset, load_clip, train_test_split
    real_ds = NpzVideoDataset(real_meshes_dir, filter_classes=ACTION_CLASSES)
    train_ds, _ = train_test_split(real_ds, train_ratio=0.8, seed=1337)
    label_dict = {cls: i for i, cls in enumerate(sorted({it.cls for it in real_ds.items}))}

    from . import stats_cache as SC
    fp = hit = None
    if stats_cache:
        fp = SC.fingerprint(train_ds.items, real_kp_dir, model_sha, compute, clip_len, stride)
        hit = SC.load(stats_cache, fp)
        if hit is not None and hit["classes"] != sorted(label_dict):
            hit = None
        if not all_agree(hit is not None):  # a miss on any rank: every rank runs the full flow
            hit = None

    if hit is not None:
        # cached: stats and centroids from the exchanged sufficient statistics; no real set, no exchange
        stats = VE.stats_from_sums(hit["stats_sums"], hit["stats_counts"], device)
        dims_raw, dims_diff = VE.infer_dims_from_stats(stats)

        def load_only():
            mp = model_path.result() if isinstance(model_path, Future) else model_path
            return VE.load_model(mp, dims_raw, dims_diff, device=device, compute=compute)

        t1 = time.perf_counter()
        model = guarded("checkpoint", load_only)
        centroids = ops.centroid_finalize(torch.from_numpy(hit["cent_sums"]).to(device),
                                          torch.from_numpy(hit["cent_counts"]).to(device))
        t2 = time.perf_counter()
    else:
        model, stats, centroids, t1, t2 = _real_set_phases(VE, ops, real_meshes_dir, model_path, real_kp_dir, clip_len,
                                                           stride, device, compute, rank, ws, train_ds, label_dict,
                                                           load_clip, stats_cache, fp)

    # phase 3: this rank's generated videos -> (ac, tc); no collective until the gather to rank 0
    def local_scores():
        combined, feats_host = {}, None
        if mine.items:
            fs = gen_fs.result() if gen_fs is not None else VE.load_frame_store(mine.items, keypoint_dir,
                                                                                 keypoint_dir is not None)
            store = ops.DeviceFrameStore.from_host(fs, device)
            feats = VE.extract_window_features(model, mine, keypoint_dir, stats, clip_len, stride, device,
                                               store=store, frame_embed=bool(save_features))
            ac = VE.compute_action_consistency_scores(feats, centroids, label_dict)
            tc = VE.compute_temporal_coherence_scores(feats, centroids, label_dict)
            combined = VE.combine_scores(ac, tc)
            if save_features:
                feats_host = {"seq_embeds": feats["seq_embeds"].cpu(), "frame_embeds": feats["frame_embeds"].cpu(),
                              "cls_names": list(feats["cls_names"]), "vid_names": list(feats["vid_names"])}
        if torch.cuda.is_available() and str(device).startswith("cuda"):
            torch.cuda.synchronize(device)
            model.status()  # a device fault in this rank's last encode stops every rank (guarded) instead of scoring
        return combined, feats_host

    combined, feats_host = guarded("generated-set scoring", local_scores)
    t3 = time.perf_counter()
    parts = gather_to_rank0(combined)
    fparts = gather_to_rank0(feats_host) if save_features else None
    if timings is not None:
        timings.update(stats_s=t1 - t0, centroids_s=t2 - t1, gen_s=t3 - t2, rank=rank, world=ws,
                       stats_cache="off" if not stats_cache else ("hit" if hit is not None else "miss"))
    if rank != 0:
        return None
    merged = merge_scores(parts)
    if out_json:
        with open(out_json, "w") as f:
            json.dump(merged, f, indent=2)
    if save_features:
        save_window_features(fparts, save_features, getattr(model, "d_model", 256))
    if human_scores_path and os.path.exists(human_scores_path):
        for key in ("ac", "tc"):
            sc = {v: e[key] for v, e in merged.items() if key in e}
            corr, p, m = VE.compute_spearman_correlation(sc, human_scores_path, key)
            if corr is not None:
                print(f"{key.upper()} Spearman: {corr:.4f} (p={p:.4e}, matched {len(m)})")
    return merged


def _real_set_phases(VE, ops, real_meshes_dir, model_path, real_kp_dir, clip_len, stride, device, compute, rank, ws,
                     train_ds, label_dict, load_clip, stats_cache=None, fp=None):
    """Phases 1-2 of the flow: the real-train shard's stats and centroid sufficient statistics, each exchanged after
    agree(); rank 0 writes the stats cache (when asked) from the exchanged sums."""
    my_train = shard(train_ds.items, rank, ws)
    # phase 1: this rank's real-train shard -> float64 stats sufficient statistics
    def local_stats():
        sums = torch.zeros((2, ops.FEAT_DIM), device=device, dtype=torch.float64)
        counts = np.zeros(2, np.int64)
        store = None
        if my_train:  # an empty shard still takes part in the exchange with zeros
            store = ops.DeviceFrameStore.from_host(VE.load_frame_store(my_train, real_kp_dir, False), device)
            ops.stats_accumulate(store, range(store.n_videos), sums, counts)
        return store, sums, counts

    real_store, sums, counts = guarded("real-set statistics", local_stats)
    s, c = stats_reduce_fn(sums, counts)
    stats = VE.stats_from_sums(s, c, device)
    dims_raw, dims_diff = VE.infer_dims_from_stats(stats)

    # phase 2: checkpoint -> encoder; this rank's real-train windows -> centroid sufficient statistics
    captured = {}

    def capture(sums_, counts_):  # the exchange happens after agree(), below
        captured["s"], captured["c"] = sums_, counts_
        return sums_, counts_

    def local_centroids():
        mp = model_path.result() if isinstance(model_path, Future) else model_path
        model = VE.load_model(mp, dims_raw, dims_diff, device=device, compute=compute)
        if real_store is not None and real_kp_dir is not None:
            for i, it in enumerate(my_train):
                if real_store.host_videos[i, 3] == 0:
                    load_clip(it, real_kp_dir, require_kp=True)  # raises like utils.py:416-417
        VE.build_real_centroids(model, real_meshes_dir, real_kp_dir, stats, clip_len, stride, device,
                                train_items=my_train, label_dict=label_dict, store=real_store, reduce_fn=capture)
        return model

    t1 = time.perf_counter()
    model = guarded("checkpoint / real-set centroids", local_centroids)
    csum, ccnt = centroid_reduce_fn(captured["s"], captured["c"])
    centroids = ops.centroid_finalize(csum, ccnt)
    t2 = time.perf_counter()
    if stats_cache and rank == 0:
        # after the exchanges: a failed write (read-only dir, full disk) only costs the cache, so it is a warning here
        # rather than an error the other ranks would wait for in the next agree()
        from . import stats_cache as SC
        try:
            SC.save(stats_cache, fp, s.cpu().numpy(), c, csum.cpu().numpy(), ccnt.cpu().numpy(), sorted(label_dict))
        except OSError as e:
            warnings.warn(f"stats cache {stats_cache!r} not written: {e}")
    return model, stats, centroids, t1, t2

def save_window_features(parts: List[Optional[dict]], path: str, d_model: int = 256) -> None:
    """window_features.pt (eval.py:197-204 layout) from the per-rank feature dicts, concatenated in rank order."""
    parts = [p for p in parts if p is not None]
    if parts:
        out = {"seq_embeds": torch.cat([p["seq_embeds"] for p in parts]),
               "frame_embeds": torch.cat([p["frame_embeds"] for p in parts]),
               "cls_names": [c for p in parts for c in p["cls_names"]],
               "vid_names": [v for p in parts for v in p["vid_names"]]}
    else:
        out = {"seq_embeds": torch.empty(0, d_model), "frame_embeds": torch.empty(0, 33, d_model), "cls_names": [],
               "vid_names": []}
    torch.save(out, path)
    print(f"Saved features to {path}")
