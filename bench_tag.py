"""TAG-Bench-shaped workload of bench.py (`--workload tag`, BASELINE.json configs[3] on pre-extracted features): the
whole eval.py flow (eval.py:350-466) over 300 generated videos of mixed length (32..128 frames = 1..13 windows each)
plus a 10-class real set, video-sharded over the ranks with the RCCL exchanges of the stats / centroid sufficient
statistics (vge.dist.run_eval_distributed): npz ingest -> ModalityStats -> real centroids -> window features ->
AC / TC -> video_scores.json on rank 0.  One step = one full flow; value = 300 videos x steps / the max-over-ranks
wall time, so it includes host ingest (npz zlib decode) and checkpoint load like the reference's eval.py does.

The dataset is written once per box by rank 0 (vge.synth.write_dataset, reference on-disk layout) under
$VGE_TAG_ROOT (default /tmp/vge_tag_bench) and reused.  The extractor stages (config 3's TokenHMR / DWPose) are
not part of this workload; their per-frame cost is measured by `--workload e2e`.
"""
from __future__ import annotations

import json
import os
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

N_GEN = 300
T_GEN = (32, 48, 64, 96, 128, 40, 72)
N_REAL_PER_CLASS, T_REAL = 8, (64, 48, 96)


def _dataset(rank: int, world: int):
    from vge import synth
    root = Path(os.environ.get("VGE_TAG_ROOT", "/tmp/vge_tag_bench"))
    spec = {"n_gen": N_GEN, "t_gen": T_GEN, "n_real": N_REAL_PER_CLASS, "t_real": T_REAL, "v": 1}
    marker = root / "spec.json"
    if rank == 0 and not (marker.exists() and json.loads(marker.read_text()) == json.loads(json.dumps(spec))):
        paths = synth.write_dataset(str(root), n_real_per_class=N_REAL_PER_CLASS, n_gen=N_GEN, T_real=T_REAL,
                                    T_gen=T_GEN, kp_short_every=7)
        synth.save_checkpoint(str(root / "model.pt"), synth.make_state_dict(synth.DIMS_RAW, synth.DIMS_DIFF))
        marker.write_text(json.dumps(spec))
    if world > 1:
        dist.barrier()
    return {"real": str(root / "real"), "real_kp": str(root / "real_kp"), "gen": str(root / "generated_meshes"),
            "gen_kp": str(root / "generated_kps"), "ckpt": str(root / "model.pt")}


def cpu_baseline(workers: int = 4):
    """oracle/evalflow.run_eval (the CPU restatement of eval.py:350-466 in the reference's structure: DataLoader
    batch_size 32 with `workers` worker processes featurising, the torch-fp32 encoder on the process's CPU share)
    over the same on-disk set, one whole flow, timed on this host.  Runs before the GPU is initialised (forked
    workers); writes the dataset first if it is missing."""
    from oracle import evalflow
    from vge import synth
    p = _dataset(0, 1)
    share = max(1, min(16, len(os.sched_getaffinity(0))))
    torch.set_num_threads(share)
    sd = synth.make_state_dict(synth.DIMS_RAW, synth.DIMS_DIFF)
    tm = {}
    t0 = time.perf_counter()
    scores, _ = evalflow.run_eval(p["real"], p["real_kp"], p["gen"], p["gen_kp"], sd, synth.DIMS_RAW, synth.DIMS_DIFF,
                                  workers=workers, timings=tm)
    dt = time.perf_counter() - t0
    return {"value": len(scores) / dt, "unit": "videos/s", "cores": share, "kind": "port",
            "sample": f"one whole flow over the same {len(scores)} generated videos ({tm.get('n_windows')} windows) + "
                      f"{N_REAL_PER_CLASS * 10} real videos: oracle/evalflow.run_eval (npz load, stats, centroids, "
                      f"DataLoader(batch_size=32, num_workers={workers}) featurising, torch-fp32 encoder on {share} "
                      f"threads, AC/TC), {dt:.1f} s wall: stats {tm.get('stats_s', 0):.1f} s, centroids "
                      f"{tm.get('centroids_s', 0):.1f} s, generated windows {tm.get('gen_extract_s', 0):.1f} s, "
                      f"metrics {tm.get('metrics_s', 0):.2f} s"}


def cpu_baseline_extract(seconds: float):
    """The end-to-end job's CPU rate: the extraction chain's per-frame cost on this host (bench_e2e.cpu_baseline_e2e:
    the fp32 torch oracles of TokenHMR, YOLOX-L + RTMPose-l and the Faster R-CNN gate on a bounded sample) over the
    set's mean frames per video; the flow's own share (cpu_baseline: ~1 % of it) is not added."""
    import bench_e2e
    r = bench_e2e.cpu_baseline_e2e(seconds, True)
    mean_t = float(np.mean([T_GEN[k % len(T_GEN)] for k in range(N_GEN)]))
    fps = r["value"] * 32.0
    return {**r, "value": fps / mean_t,
            "sample": r["sample"].replace("/ 32 frames per clip", f"/ {mean_t:.1f} frames per video (the set's mean)")}


def run(args, world, rank, dev, metric, cpu=None):
    from vge.dist import run_eval_distributed
    t0 = time.perf_counter()
    p = _dataset(rank, world)
    setup_s = time.perf_counter() - t0

    def flow(tm=None):
        return run_eval_distributed(p["gen"], p["real"], p["ckpt"], p["gen_kp"], p["real_kp"], out_json=None,
                                    device=dev, compute=args.compute, timings=tm)

    for _ in range(args.warmup):
        flow()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    tm = {}
    t = time.perf_counter()
    for _ in range(args.steps):
        scores = flow(tm)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t
    if world > 1:
        dt_t = torch.tensor([dt], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
        dt = float(dt_t.item())
    if rank != 0:
        return None
    assert scores is not None and len(scores) == N_GEN
    vals = np.array([[v.get("ac", np.nan), v["tc"]] for v in scores.values()], np.float64)
    assert np.isfinite(vals[:, 1]).all()
    return {
        "metric": metric,
        "value": N_GEN * args.steps / dt,
        "unit": "videos/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": args.compute,
        "data": "synthetic TAG-Bench-shaped set (vge.synth.write_dataset: 300 generated videos of 32-128 frames, "
                "10 x 8 real videos, every 7th keypoint file shorter than its mesh sequence), random-init weights",
        "config": {"workload": "BASELINE config 4 on pre-extracted features: the full eval.py flow (npz ingest, "
                               "ModalityStats, real centroids with RCCL all-gather of the sufficient statistics, "
                               "window features, AC/TC, scores gathered to rank 0)",
                   "videos": N_GEN, "parallelism": f"video-sharded x{world}"},
        "stage_s_last_step_rank0": {k: v for k, v in tm.items() if k.endswith("_s")},
        "setup_s": setup_s,
        "roofline": None,   # host-bound flow (npz inflate, checkpoint read): stage_s_last_step_rank0 has the split
        "cpu_baseline": cpu,
    }


def run_extract(args, world, rank, dev, metric, cpu=None):
    """BASELINE config 4 END TO END as one video-sharded job (`bench.py --workload tag --extract`): the TAG-Bench-shaped
    generated set (300 videos of 32-128 frames, 256x256 RGB frames resident in HBM) goes through the extraction chain
    on each rank's contiguous shard -- detectron2 Faster R-CNN X101-32x8d-FPN gate + TokenHMR (ViT-H/16 + decoder),
    YOLOX-L + DWPose (RTMPose-l), vge.extract.extract_videos: passes of up to 1,024 frames packing several videos, the
    single-person gate and 80 % rule per video, npz of the kept frames and keypoints.npy of every frame written in the
    reference's generated-set layout (extract_mesh.py:150-241, process_video.py:59-94) -- then, after a barrier, the
    video-sharded eval flow over the written files (vge.dist.run_eval_distributed: eval.py:350-466, ModalityStats and
    real-class centroids from the pre-extracted real set with their sufficient statistics all-gathered, scores
    gathered to rank 0).  One step = extraction + flow; value = 300 videos x steps / the max-over-ranks wall time.  The
    frames are drawn at setup from a pool of synthetic scenes by what the gate detector finds in each (9 videos in 10
    pass the gate with 1-3 non-single-person frames; 1 in 10 is rejected), as bench_e2e.py does; every step runs both
    detectors on every frame again and takes every decision from their output."""
    import shutil
    from vge import synth
    from vge.dist import run_eval_distributed, shard
    from vge.dwpose import RTMPOSE_L, YOLOX_L, DwposeExtractor, Wholebody, YoloxDetector
    from vge.extract import extract_videos, gate_mask
    from vge.frcnn import FRCNN_X101, FrcnnDetector
    from vge.hmr import TOKENHMR, HmrExtractor
    t0 = time.perf_counter()
    p = _dataset(rank, world)
    root = Path(os.environ.get("VGE_TAG_ROOT", "/tmp/vge_tag_bench")) / "e2e"
    gen, gkp = root / "generated_meshes", root / "generated_kps"
    FC = 1024
    hmr = HmrExtractor(synth.make_hmr_state_dict(TOKENHMR), TOKENHMR, device=dev, max_frames=FC)
    gdet = FrcnnDetector(synth.make_gate_frcnn_state_dict(FRCNN_X101), FRCNN_X101, device=dev, chunk=128)
    wb = Wholebody(YoloxDetector(synth.make_gate_detector_state_dict(YOLOX_L), YOLOX_L, device=dev, chunk=256),
                   DwposeExtractor(synth.make_rtmpose_state_dict(RTMPOSE_L), RTMPOSE_L, device=dev, max_instances=2 * FC))
    pool = torch.from_numpy(synth.make_frame_pool(7000, 2048)).to(dev)
    one = gate_mask(gdet.detect(pool)["n_person"].cpu().numpy())
    good, bad = np.flatnonzero(one), np.flatnonzero(~one)
    if good.size < 256 or bad.size < 64:
        raise RuntimeError(f"tag --extract: the gate detector finds one person in {good.size} of 2048 pool frames")
    rs = np.random.default_rng(23)   # the same plan on every rank: a video's frames do not depend on the world size
    plan = []
    for k in range(N_GEN):
        T = T_GEN[k % len(T_GEN)]
        nb = int(np.ceil(0.3 * T)) if k % 10 == 9 else 1 + k % 3
        plan.append((synth.generated_name(k), rs.permutation(np.concatenate([rs.choice(bad, nb), rs.choice(good, T - nb)]))))
    mine = shard(plan, rank, world)
    frames = [(s, pool[torch.from_numpy(i).to(dev)].contiguous()) for s, i in mine]
    del pool
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t0
    n_frames = sum(int(f.shape[0]) for _, f in frames)

    def step(tm):
        if rank == 0:
            shutil.rmtree(root, ignore_errors=True)
        if world > 1:
            dist.barrier()
        t = time.perf_counter()
        wrote = extract_videos(hmr, wb, gdet, frames, gen, gkp, max_frames=FC)
        torch.cuda.synchronize()
        tm["extract_s"] = time.perf_counter() - t
        if world > 1:
            dist.barrier()   # every shard's files are written before any rank scans the generated set
        t = time.perf_counter()
        scores = run_eval_distributed(str(gen), p["real"], p["ckpt"], str(gkp), p["real_kp"], out_json=None,
                                      device=dev, compute=args.compute, timings=tm)
        tm["flow_s"] = time.perf_counter() - t
        return scores, wrote

    tm = {}
    for _ in range(args.warmup):
        step(tm)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.steps):
        scores, wrote = step(tm)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t
    if world > 1:
        dt_t = torch.tensor([dt], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
        dt = float(dt_t.item())
    if rank != 0:
        return None
    accepted = sum(1 for v in wrote.values() if v)
    return {
        "metric": metric,
        "value": N_GEN * args.steps / dt,
        "unit": "videos/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": f"bf16 (extractors: bf16 operands, f32 accumulate) + {args.compute} (scorer)",
        "data": "synthetic TAG-Bench-shaped set: 300 generated videos of 32-128 frames as 256x256 RGB frames in HBM "
                "(drawn from vge.synth.make_frame_pool by the gate detector's findings), 10 x 8 pre-extracted real "
                "videos; random-init weights of the Faster R-CNN X101-32x8d-FPN, TokenHMR, YOLOX-L, RTMPose-l and "
                "scorer architectures",
        "config": {"workload": "BASELINE config 4 end to end: each rank extracts its shard of the generated videos "
                               "(gate detector + TokenHMR, YOLOX-L + DWPose -> npz / keypoints.npy on disk), then the "
                               "video-sharded eval.py flow over the written files (stats / centroid sufficient "
                               "statistics all-gathered, scores gathered to rank 0)",
                   "videos": N_GEN, "frames_rank0": n_frames, "parallelism": f"video-sharded x{world}"},
        "rank0_last_step": {"extract_s": tm.get("extract_s"), "flow_s": tm.get("flow_s"),
                            "videos_extracted": len(wrote), "videos_accepted": accepted,
                            "frames_per_s_extract": n_frames / tm["extract_s"] if tm.get("extract_s") else None},
        "videos_scored": len(scores) if scores is not None else None,
        "setup_s": setup_s,
        "roofline": None,   # the extractors' and scorer's kernels are measured by the e2e / score workloads
        "cpu_baseline": cpu,
    }
