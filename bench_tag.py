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
