"""The scoring driver: eval.py's flow (reference eval.py:350-466) on libvge.

Same function names, argument meaning and outputs as the reference:
  load_model                          eval.py:136-165   (torch.load(weights_only=True); plain state_dict or
                                                         {model_state_dict|state_dict, d_model, ...}; a missing
                                                         key is an error here -- see INTEGRATION.md)
  compute_stats_from_npz              utils.py:595-801  (HIP featurise in stats mode + float64 column sums)
  build_real_centroids                eval.py:260-286   (+ build_train_centroids_subset utils.py:1018-1045)
  extract_window_features             eval.py:168-206
  compute_action_consistency_scores   eval.py:229-257
  compute_temporal_coherence_scores   eval.py:209-226
  compute_spearman_correlation        eval.py:297-347
  run_eval                            eval.py:350-454 (writes video_scores.json)
Per-frame features are decoded on the host (npz/zlib, libvge's native multithreaded decoder) into a
frame store that lives in HBM; every numeric step after that runs in the HIP kernels of libvge.so.
"""
from __future__ import annotations

import json
import os
import time
from collections import defaultdict
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import ops
from .data import (ACTION_CLASSES, FrameStore, NpzVideoDataset, VideoItem, _canonicalize_class,
                   create_dataset_from_generated_meshes, enumerate_test_windows, load_clip, pack_frame_store,
                   sample_all_windows_npz, train_test_split)


# ----------------------------------------------------------------------------- loading

def load_frame_store(items: Sequence[VideoItem], keypoint_dir: Optional[str], require_kp: bool,
                     workers: int = 0) -> FrameStore:
    """Decode the npz + keypoints.npy of `items` into a frame store (pinned host memory when a GPU is
    present): libvge's native multithreaded decoder (vge/ingest.py, include/vge_ingest.h)."""
    from .ingest import load_frame_store_native
    return load_frame_store_native(items, keypoint_dir, require_kp, threads=workers)


def load_frame_store_numpy(items: Sequence[VideoItem], keypoint_dir: Optional[str], require_kp: bool,
                           workers: int = 8) -> FrameStore:
    """The np.load reader (the reference's own, utils.py:383-424) in a thread pool: kept as the ingest
    baseline of tools/ingest_bench.py."""
    with ThreadPoolExecutor(max_workers=max(1, workers)) as ex:
        clips = list(ex.map(lambda it: load_clip(it, keypoint_dir, require_kp), items))
    return pack_frame_store(clips, [it.name for it in items], [it.cls for it in items])


class ModalityStatsGPU:
    """mean/std f32 on device in feats column order ([2596], or [2356] for the keypoint-less layout) + the float64
    sufficient statistics ([2,2596] sums, frame counts).  The layout follows compute_stats_from_npz: keypoint stats
    exist iff some real-train keypoint frame was read (utils.py:753-755), and infer_dims_from_stats then gives the
    model 5 or 4 modalities (eval.py:119-123)."""

    def __init__(self, mean, std, sums, counts, layout="kp"):
        self.mean, self.std, self.sums, self.counts, self.layout = mean, std, sums, counts, layout


def stats_layout(counts) -> str:
    """'kp' iff keypoint frames were counted (the reference's n_kp_raw > 0), else the keypoint-less 'nokp'."""
    return "kp" if int(counts[1]) > 0 else "nokp"


def compute_stats_from_npz(train_items: Sequence[VideoItem], keypoint_dir: str, device="cuda",
                           store: Optional[ops.DeviceFrameStore] = None, reduce_fn=None) -> ModalityStatsGPU:
    """utils.py:595-801.  `reduce_fn(sums, counts)` (optional) all-reduces the sufficient statistics
    across ranks before finalising (sharded real set)."""
    assert len(train_items) > 0, "compute_stats_from_npz: train_items is empty"
    if store is None:
        store = ops.DeviceFrameStore.from_host(load_frame_store(train_items, keypoint_dir, require_kp=False), device)
    sums = torch.zeros((2, ops.FEAT_DIM), device=device, dtype=torch.float64)
    counts = np.zeros(2, np.int64)
    ops.stats_accumulate(store, range(store.n_videos), sums, counts)
    if reduce_fn is not None:
        sums, counts = reduce_fn(sums, counts)
    layout = stats_layout(counts)
    mean, std = ops.stats_finalize(sums, counts, layout)
    return ModalityStatsGPU(mean, std, sums, counts, layout)


def _load_state_dict(model_path: str):
    ck = torch.load(model_path, map_location="cpu", weights_only=True)
    hp = {"d_model": 256, "latent_dim": 128, "time_layers": 4, "time_heads": 8, "dropout": 0.1}
    if isinstance(ck, dict):
        for k in hp:
            if k in ck and not isinstance(ck[k], torch.Tensor):
                hp[k] = ck[k]
    if isinstance(ck, dict) and "model_state_dict" in ck:
        sd = ck["model_state_dict"]
    elif isinstance(ck, dict) and "state_dict" in ck:
        sd = ck["state_dict"]
    else:
        sd = ck
    sd = {k: v.detach().float().cpu().numpy() for k, v in sd.items() if isinstance(v, torch.Tensor)}
    return sd, hp


def load_model(model_path, dims_map_raw=None, dims_map_diff=None, device="cuda", compute="f32x3") -> ops.Encoder:
    """eval.py:136-165 -> a libvge encoder handle (weights repacked into HBM).  dims: the five-modality layout or
    its keypoint-less first four (infer_dims_from_stats); anything else is VGE_ERR_UNSUPPORTED."""
    n_mod = 5
    if dims_map_raw is not None:
        n_mod = len(dims_map_raw)
        ok = n_mod in (4, 5) and list(dims_map_raw) == list(ops.MODALITIES[:n_mod]) and \
            list(dims_map_diff) == list(ops.MODALITIES[:n_mod]) and \
            tuple(dims_map_raw.values()) == ops.DIMS_RAW[:n_mod] and tuple(dims_map_diff.values()) == ops.DIMS_DIFF[:n_mod]
        if not ok:
            from .lib import UnsupportedModelError
            raise UnsupportedModelError(f"unsupported modality dims {dims_map_raw} / {dims_map_diff} (the kernels "
                                        f"are built for the five-modality layout and its keypoint-less four; "
                                        f"VGE_ERR_UNSUPPORTED)")
    if isinstance(model_path, dict):
        # a bare state dict takes the reference's defaults (eval.py:139-143: checkpoint.get("d_model", 256), 4 layers,
        # 8 heads), exactly as the same dict saved to a .pt file does (_load_state_dict); a checkpoint of another
        # shape passes its hyper-parameters: (state_dict, {"d_model": .., "time_layers": .., "time_heads": ..})
        sd = model_path
        hp = {"d_model": 256, "time_layers": 4, "time_heads": 8}
    elif isinstance(model_path, tuple):  # (state_dict, hyper-parameters) as _load_state_dict returns them
        sd, hp = model_path
    else:
        sd, hp = _load_state_dict(model_path)
    if (int(hp["d_model"]), int(hp["time_heads"])) != (ops.D_MODEL, 8) and compute != "f32":
        # the tiled 3xfp16 / fp16 kernels are built for d_model 256 x 8 heads; other checkpoint shapes run on the
        # generic exact-f32 kernels (vge_encoder_gen.hip)
        compute = "f32"
    return ops.Encoder(sd, time_layers=int(hp["time_layers"]), time_heads=int(hp["time_heads"]),
                       d_model=int(hp["d_model"]), device=device, compute=compute, n_modalities=n_mod)


def infer_dims_from_stats(stats) -> Tuple[Dict[str, int], Dict[str, int]]:
    """eval.py:104-133: vit, global, pose, beta, plus kp2d when the stats hold keypoint statistics."""
    n = ops.N_MODALITIES[getattr(stats, "layout", "kp")]
    return dict(zip(ops.MODALITIES[:n], ops.DIMS_RAW[:n])), dict(zip(ops.MODALITIES[:n], ops.DIMS_DIFF[:n]))


# ----------------------------------------------------------------------------- windows -> embeddings

def _window_tensor(samples, name_to_idx, device):
    w = np.array([[name_to_idx[it.path], s] for it, s in samples], np.int32).reshape(-1, 2)
    return torch.from_numpy(w).to(device)


def encode_windows(model: ops.Encoder, store: ops.DeviceFrameStore, windows: torch.Tensor, stats: ModalityStatsGPU,
                   batch: int = 1024, frame_embed: bool = False):
    """featurise + encode windows in batches; returns (seq [N,d], frame [N,33,d] | None, tc [N]), d = d_model."""
    n = int(windows.shape[0])
    dev = windows.device
    if model.layout != stats.layout:
        raise ValueError(f"model takes the {model.layout!r} feature layout but the stats are {stats.layout!r} "
                         f"(the reference would fail on the feature width)")
    d = getattr(model, "d_model", ops.D_MODEL)
    seq = torch.empty((n, d), device=dev)
    tcw = torch.empty((n,), device=dev)
    fe = torch.empty((n, 33, d), device=dev) if frame_embed else None
    model.reserve(min(batch, max(n, 1)))
    feats = torch.empty((min(batch, max(n, 1)), 32, model.feat_dim), device=dev)
    for b0 in range(0, n, batch):
        b1 = min(n, b0 + batch)
        f = ops.featurize(store, windows[b0:b1], stats.mean, stats.std, out=feats[: b1 - b0], layout=stats.layout)
        s, fr, t = model.encode(f, frame_embed=frame_embed, tc=True)
        seq[b0:b1] = s
        tcw[b0:b1] = t
        if frame_embed:
            fe[b0:b1] = fr
    # the conv kernel's device status word: a fault in the last (or only) batch has no later vge_encode to report it,
    # so check it once every launch has completed, before the caller consumes these embeddings
    torch.cuda.synchronize(dev)
    model.status()
    return seq, fe, tcw


def build_real_centroids(model: ops.Encoder, real_meshes_dir: str, real_kp_dir: str, stats: ModalityStatsGPU,
                         clip_len: int = 32, stride: int = 8, device="cuda", train_items=None, label_dict=None,
                         store: Optional[ops.DeviceFrameStore] = None, reduce_fn=None):
    """eval.py:260-286 / utils.py:1018-1045 -> (centroids [C,256] device, label_dict, counts)."""
    if train_items is None or label_dict is None:
        real_ds = NpzVideoDataset(real_meshes_dir, filter_classes=ACTION_CLASSES)
        train_ds, _ = train_test_split(real_ds, train_ratio=0.8, seed=1337)
        train_items = train_ds.items
        label_dict = {cls: i for i, cls in enumerate(sorted({it.cls for it in real_ds.items}))}
    C_ = len(label_dict)
    sums = torch.zeros((C_, getattr(model, "d_model", ops.D_MODEL)), device=device)
    counts = torch.zeros((C_,), device=device)
    if len(train_items):
        samples = enumerate_test_windows(NpzVideoDataset("", items=list(train_items)), clip_len, stride)
        if store is None:
            store = ops.DeviceFrameStore.from_host(load_frame_store(train_items, real_kp_dir,
                                                                    require_kp=real_kp_dir is not None), device)
        idx = {it.path: i for i, it in enumerate(train_items)}
        win = _window_tensor(samples, idx, device)
        seq, _, _ = encode_windows(model, store, win, stats)
        y = torch.as_tensor([label_dict[it.cls] for it, _ in samples], dtype=torch.int32, device=device)
        ops.centroid_accumulate(seq, y, sums, counts)
    if reduce_fn is not None:
        sums, counts = reduce_fn(sums, counts)
    return ops.centroid_finalize(sums, counts), label_dict, counts


def extract_window_features(model: ops.Encoder, dataset: NpzVideoDataset, keypoint_dir: str, stats: ModalityStatsGPU,
                            clip_len: int = 32, stride: int = 8, device="cuda", frame_embed: bool = False,
                            store: Optional[ops.DeviceFrameStore] = None, save_path: Optional[str] = None):
    """eval.py:168-206 over all windows of `dataset` (sample_all_windows_npz order).  save_path: torch.save of
    {seq_embeds [Nw,256], frame_embeds [Nw,33,256], cls_names, vid_names} on the CPU like eval.py:197-204
    (frame embeddings are then produced too)."""
    if ops.layout_of(keypoint_dir) != stats.layout:
        # the reference fails here too: a keypoint-less WindowDataset's rows (2356) do not broadcast against kp stats
        # (2596), and a keypoint dir with keypoint-less stats finds keypoints_raw_mean None (utils.py:406-425, 496-514)
        raise ValueError(f"generated keypoint dir {keypoint_dir!r} gives the {ops.layout_of(keypoint_dir)!r} feature "
                         f"layout but the real-set stats are {stats.layout!r}: pass both keypoint dirs or neither")
    samples = sample_all_windows_npz(dataset, clip_len, stride)
    if store is None:
        store = ops.DeviceFrameStore.from_host(load_frame_store(dataset.items, keypoint_dir,
                                                                require_kp=keypoint_dir is not None), device)
    idx = {it.path: i for i, it in enumerate(dataset.items)}
    win = _window_tensor(samples, idx, device)
    seq, fe, tcw = encode_windows(model, store, win, stats, frame_embed=frame_embed or bool(save_path))
    out = {"seq_embeds": seq, "frame_embeds": fe, "tc_window": tcw,
           "cls_names": [it.cls for it, _ in samples], "vid_names": [it.name for it, _ in samples]}
    if save_path:
        torch.save({"seq_embeds": seq.cpu(), "frame_embeds": fe.cpu(), "cls_names": list(out["cls_names"]),
                    "vid_names": list(out["vid_names"])}, save_path)
        print(f"Saved features to {save_path}")
    return out


# ----------------------------------------------------------------------------- metrics

def _video_index(features):
    vids, first = [], []
    for i, v in enumerate(features["vid_names"]):
        vid = os.path.splitext(v)[0]
        if not vids or vids[-1] != vid:
            vids.append(vid)
            first.append(i)
    first.append(len(features["vid_names"]))
    return vids, first


def _score(features, centroids, label_dict):
    if "_scores" in features:
        return features["_scores"]
    dev = features["seq_embeds"].device
    vids, first = _video_index(features)
    if len(set(vids)) != len(vids):
        raise ValueError("windows of one video must be contiguous (sample_all_windows_npz order)")
    vcls = []
    for k in range(len(vids)):
        c = _canonicalize_class(features["cls_names"][first[k]])
        vcls.append(label_dict[c] if (label_dict is not None and c in label_dict and
                                      centroids is not None and label_dict[c] < len(centroids)) else -1)
    tcw = features["tc_window"]
    if tcw is None:
        tcw = ops.tc_windows(features["frame_embeds"])
    ac, tc = ops.score_videos(features["seq_embeds"], tcw,
                              torch.as_tensor(first, dtype=torch.int32, device=dev),
                              torch.as_tensor(vcls, dtype=torch.int32, device=dev), centroids)
    ac = ac.cpu().numpy()
    tc = tc.cpu().numpy()
    features["_scores"] = (vids, vcls, ac, tc)
    return features["_scores"]


def compute_action_consistency_scores(features, centroids, label_dict) -> Dict[str, float]:
    vids, vcls, ac, _ = _score(features, centroids, label_dict)
    return {v: float(ac[k]) for k, v in enumerate(vids) if vcls[k] >= 0}


def compute_temporal_coherence_scores(features, centroids=None, label_dict=None) -> Dict[str, float]:
    vids, _, _, tc = _score(features, centroids, label_dict)
    return {v: float(tc[k]) for k, v in enumerate(vids)}


def combine_scores(ac: Dict[str, float], tc: Dict[str, float]) -> Dict[str, dict]:
    out = {}
    for v in sorted(set(ac) | set(tc)):
        e = {}
        if v in ac:
            e["ac"] = ac[v]
        if v in tc:
            e["tc"] = tc[v]
        out[v] = e
    return out


def _norm_name(name: str) -> str:
    stem = os.path.splitext(os.path.basename(name))[0]
    return stem.replace("_videos_", "_").replace("videos_", "").replace("_video_", "_")


def compute_spearman_correlation(model_scores: dict, human_scores_path: str, human_key: str):
    """eval.py:297-347 (sign-inverted Spearman; exact then suffix name matching)."""
    from scipy.stats import spearmanr
    with open(human_scores_path) as f:
        human = json.load(f)
    by_name = {_norm_name(k): v for k, v in model_scores.items()}
    mv, hv, matched = [], [], []
    for hname, hdata in human.items():
        if human_key not in hdata:
            continue
        hn = _norm_name(hname)
        if hn in by_name:
            mv.append(by_name[hn])
            hv.append(hdata[human_key])
            matched.append((hn, hname))
            continue
        hp = hn.split("_")
        for mn, ms in by_name.items():
            mp = mn.split("_")
            if len(mp) >= 2 and len(hp) >= 2 and (mp[-2:] == hp[-2:] or mp[-1] == hp[-1]):
                mv.append(ms)
                hv.append(hdata[human_key])
                matched.append((mn, hname))
                break
    if len(mv) < 2:
        print(f"Warning: Only {len(mv)} matched videos for {human_key}. Need at least 2.")
        return None, None, matched
    corr, p = spearmanr(np.array(mv), np.array(hv))
    if corr is not None and not np.isnan(corr):
        corr = -float(corr)
    return corr, p, matched


def stats_from_sums(sums, counts, device) -> ModalityStatsGPU:
    """ModalityStats from (exchanged or cached) sufficient statistics: vge_stats_finalize on the device."""
    sums = torch.as_tensor(sums, dtype=torch.float64).to(device)
    counts = np.asarray(counts, np.int64)
    layout = stats_layout(counts)
    mean, std = ops.stats_finalize(sums, counts, layout)
    return ModalityStatsGPU(mean, std, sums, counts, layout)


def run_eval(generated_meshes_dir: str, real_meshes_dir: str, model_path, keypoint_dir: str, real_kp_dir: str,
             human_scores_path: Optional[str] = None, clip_len: int = 32, stride: int = 8,
             out_json: Optional[str] = "video_scores.json", device="cuda", timings: Optional[dict] = None,
             compute: str = "f32x3", save_features: Optional[str] = None, stats_cache: Optional[str] = None):
    """eval.py __main__ (350-466) on one GPU; returns the combined {video: {ac, tc}} dict.  save_features: the
    window_features.pt of eval.py:439-443 (off by default: it copies every frame embedding to the host).
    stats_cache: path of the real set's stats + centroid artifact (vge/stats_cache.py): read when its fingerprint
    matches (the real set is then neither decoded nor encoded), else computed and written."""
    from . import stats_cache as SC
    t0 = time.perf_counter()
    real_ds = NpzVideoDataset(real_meshes_dir, filter_classes=ACTION_CLASSES)
    train_ds, _ = train_test_split(real_ds, train_ratio=0.8, seed=1337)
    label_dict = {cls: i for i, cls in enumerate(sorted({it.cls for it in real_ds.items}))}
    fp = hit = None
    if stats_cache:
        fp = SC.fingerprint(train_ds.items, real_kp_dir, SC.model_digest(model_path), compute, clip_len, stride)
        hit = SC.load(stats_cache, fp)
        if hit is not None and hit["classes"] != sorted(label_dict):
            hit = None
    if hit is not None:
        stats = stats_from_sums(hit["stats_sums"], hit["stats_counts"], device)
        dims_raw, dims_diff = infer_dims_from_stats(stats)
        model = load_model(model_path, dims_raw, dims_diff, device=device, compute=compute)
        t1 = time.perf_counter()
        centroids = ops.centroid_finalize(torch.from_numpy(hit["cent_sums"]).to(device),
                                          torch.from_numpy(hit["cent_counts"]).to(device))
    else:
        real_store = ops.DeviceFrameStore.from_host(load_frame_store(train_ds.items, real_kp_dir, require_kp=False),
                                                    device)
        stats = compute_stats_from_npz(train_ds.items, real_kp_dir, device=device, store=real_store)
        dims_raw, dims_diff = infer_dims_from_stats(stats)
        model = load_model(model_path, dims_raw, dims_diff, device=device, compute=compute)
        t1 = time.perf_counter()
        # centroids need every real-train keypoint file (WindowDataset raises otherwise)
        for i, it in enumerate(train_ds.items):
            if real_kp_dir is not None and real_store.host_videos[i, 3] == 0:
                load_clip(it, real_kp_dir, require_kp=True)  # raises FileNotFoundError like utils.py:416-417
        cap = {}

        def capture(s_, c_):
            cap["s"], cap["c"] = s_, c_
            return s_, c_

        centroids, label_dict, _ = build_real_centroids(model, real_meshes_dir, real_kp_dir, stats, clip_len, stride,
                                                        device, train_items=train_ds.items, label_dict=label_dict,
                                                        store=real_store, reduce_fn=capture)
        if stats_cache:
            SC.save(stats_cache, fp, stats.sums.cpu().numpy(), stats.counts, cap["s"].cpu().numpy(),
                    cap["c"].cpu().numpy(), sorted(label_dict))
    t2 = time.perf_counter()
    dataset = create_dataset_from_generated_meshes(generated_meshes_dir)
    feats = extract_window_features(model, dataset, keypoint_dir, stats, clip_len, stride, device,
                                    save_path=save_features)
    ac = compute_action_consistency_scores(feats, centroids, label_dict)
    tc = compute_temporal_coherence_scores(feats, centroids, label_dict)
    combined = combine_scores(ac, tc)
    torch.cuda.synchronize(device)
    t3 = time.perf_counter()
    if out_json:
        with open(out_json, "w") as f:
            json.dump(combined, f, indent=2)
    if human_scores_path and os.path.exists(human_scores_path):
        for key, sc in (("ac", ac), ("tc", tc)):
            corr, p, m = compute_spearman_correlation(sc, human_scores_path, key)
            if corr is not None:
                print(f"{key.upper()} Spearman: {corr:.4f} (p={p:.4e}, matched {len(m)})")
    if timings is not None:
        timings.update(stats_s=t1 - t0, centroids_s=t2 - t1, gen_s=t3 - t2, n_windows=len(feats["vid_names"]),
                       stats_cache="off" if not stats_cache else ("hit" if hit is not None else "miss"))
    return combined


def main(argv=None):
    """Command line of eval.py (its __main__ hard-codes the paths; here they are arguments).  Under torchrun
    (WORLD_SIZE > 1) the flow is sharded over the ranks (vge.dist.run_eval_distributed, RCCL)."""
    import argparse
    ap = argparse.ArgumentParser(description="AC / TC scores of generated videos (MI355X)")
    ap.add_argument("--generated-meshes", required=True)
    ap.add_argument("--real-meshes", required=True)
    ap.add_argument("--model", required=True, help="checkpoint with model_state_dict (eval.py:136-165)")
    ap.add_argument("--keypoints", default=None,
                    help="generated keypoint dir (<stem>/keypoints.npy); omit both keypoint dirs for the "
                         "keypoint-less 4-modality layout (keypoint_dir None)")
    ap.add_argument("--real-keypoints", default=None)
    ap.add_argument("--kp-layout", default=None, choices=["auto", "flat", "per_class"],
                    help="layout of --keypoints: auto = the reference's name sniffing (utils.py:410-417), flat = "
                         "<dir>/<stem>/keypoints.npy, per_class = <dir>/<Class>/<stem>/keypoints.npy "
                         "(default: VGE_KP_LAYOUT or auto)")
    ap.add_argument("--real-kp-layout", default=None, choices=["auto", "flat", "per_class"],
                    help="layout of --real-keypoints (as --kp-layout)")
    ap.add_argument("--human-scores", default=None)
    ap.add_argument("--out", default="video_scores.json")
    ap.add_argument("--save-features", default=None, help="e.g. window_features.pt")
    ap.add_argument("--clip-len", type=int, default=32)
    ap.add_argument("--stride", type=int, default=8)
    ap.add_argument("--compute", default="f32x3", choices=["f32x3", "f32", "f16"])
    ap.add_argument("--stats-cache", default=None,
                    help="real-set stats + centroid artifact (.npz): reused when its fingerprint matches, else written")
    a = ap.parse_args(argv)
    if (a.keypoints is None) != (a.real_keypoints is None):
        ap.error("--keypoints and --real-keypoints go together (both: the 5-modality layout; neither: keypoint-less)")
    from .data import set_keypoint_layout
    for layout, d in ((a.kp_layout, a.keypoints), (a.real_kp_layout, a.real_keypoints)):
        if layout is not None:
            if d is None:
                ap.error("a keypoint layout was given without its keypoint directory")
            set_keypoint_layout(layout, d)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        import torch.distributed as dist
        from .dist import run_eval_distributed
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        try:
            res = run_eval_distributed(a.generated_meshes, a.real_meshes, a.model, a.keypoints, a.real_keypoints,
                                       a.clip_len, a.stride, out_json=a.out, device=f"cuda:{local}",
                                       compute=a.compute, human_scores_path=a.human_scores,
                                       save_features=a.save_features, stats_cache=a.stats_cache)
        finally:
            dist.destroy_process_group()
    else:
        res = run_eval(a.generated_meshes, a.real_meshes, a.model, a.keypoints, a.real_keypoints, a.human_scores,
                       a.clip_len, a.stride, out_json=a.out, compute=a.compute, save_features=a.save_features,
                       stats_cache=a.stats_cache)
    if res is not None:
        print(f"Saved AC/TC scores for {len(res)} videos to {a.out}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
