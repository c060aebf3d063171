#!/usr/bin/env python3
"""AC/TC scoring throughput on MI355X -- BASELINE.json's metric on its configs[1] workload.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (config 2 of BASELINE.json, "1 MI355X bf16"): 256 synthetic 32-frame clips per GPU with
pre-extracted per-frame features (SMPL rotations, betas, 1024-d token, 120-d keypoints) resident in
HBM.  One step = featurise all windows (HIP) -> HumanActionScorer forward (MFMA) -> per-video AC + TC
(HIP reductions) -> scores copied to pinned host memory, in that order on one stream (--pipeline serial, the default
since round 5: the featurise no longer shares the CUs with the transformer, which then runs ~10 % faster, 0.262 vs
0.288-0.290 ms, for 185.0k-185.4k vs 183.3k-185.0k videos/s, same box, profiles/ab_r05ae_pipeline.json).
--pipeline side3: each chunk's featurise is issued on a side stream once the previous encode's conv stage has consumed
the feats buffer (vge_encoder_wait_conv), so it overlaps that chunk's fusion + transformer, and the per-video scores +
host copies run on that side stream too, launched after the next step's conv stage and featurise, with the encodes
alternating between two output buffers (side2: the scores right after the transformer); every step's work, the last
step's scores included, stays inside the timed region in every mode.  ModalityStats and the real-class centroids
(the real set is sharded over ranks, sufficient statistics all-gathered over RCCL) are built once in
the setup phase (`setup_s`).  Weak scaling: every rank scores its own 256 clips; no collective in the
step.  Compute mode: `f32x3` (3xfp16 split-precision MFMA: f32-class results, the reference computes in fp32;
|dAC|, |dTC| vs the oracle over every clip of the step are in `precision`), with the fp16-operand throughput
mode (`f16`: VGE_F16, fp16 MFMA conv encoders) run on the same workload and reported nested as
`throughput_mode` with its own precision.

Rank 0 prints ONE JSON line.  `roofline` is for the dominant kernel (the 10 MovementConvEncoders,
MFMA-bound): achieved = its algorithmic FLOPs per launch (1.7622 GFLOP per window)
/ its average duration from hipEvents recorded around it on its stream inside the timed steps (every --event-every-th
step, default 5: each event is a queue marker); peak =
the MFMA ceiling of the compute mode from rocminfo (CUs x max clock: f16 dense 4096 FLOP/clk/CU, 2516.6 TF on
MI355X; 3xfp16 split: / 3 = 838.9 TF; exact f32 256 FLOP/clk/CU, 157.3 TF; `peak_source`).  `traffic` = HBM bytes per launch from the committed PMC pass
(profiles/pmc_conv_encoder.json, FETCH_SIZE x2 + WRITE_SIZE per the guide), reported only when that pass
was taken on this tree's kernel sources, else null.  `cpu_baseline` is the oracle CPU restatement of
eval.py in the reference's structure (DataLoader workers=4, bs 32, torch-fp32 on the CPU share) timed on
this host on a bounded sample before the GPU is touched.  `--workload cfg5` runs config 5 (10k 64-frame
clips, strong scaling); `tag` config 4's flow; `e2e` config 3.

At N = 1 the default line also carries `e2e`: BASELINE config 3 (1k clips x 32 frames at 256x256: the Faster R-CNN
gate + TokenHMR and YOLOX + DWPose extractors -> featurise -> encoder -> AC/TC; bench_e2e.py) as one timed step after
one warm-up, run in a child process after the config-2 measurements, with its own stage_ms, the ViT-H GEMM and gate
detector rooflines, PMC traffic and CPU baseline (`--no-e2e` skips it).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "video-gen-evals_amd"))
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = json.loads((ROOT / "BASELINE.json").read_text())["metric"]
CLIP_LEN = 32
# algorithmic FLOPs of conv_encoder_kernel per 32-frame window: stems (K = sum of the 10 input dims =
# 2596) + 80 dilated k=5 convs 256->256 + 10 proj 256->256, 2 FLOP per MAC
CONV_FLOP_PER_WINDOW = 2 * 32 * 256 * 2596 + 80 * 2 * 32 * 256 * 256 * 5 + 10 * 2 * 32 * 256 * 256
ENCODER_FLOP_PER_WINDOW = 2.0203e9          # FlopCounterMode on model.py at T=32
F32_MFMA_PEAK_TFLOPS = 157.3                # MI355X_MICROARCH.md: v_mfma_f32_* = FP32 vector peak
# dense F16 MFMA peak: 256 CUs x 4 SIMDs x 1024 FLOP/clk x 2.4 GHz (MI355X_MICROARCH.md "~2.5 PF dense");
# the 3xfp16 path issues 3 f16 MFMAs per f32 product, so its ceiling in algorithmic f32 FLOP/s is 1/3 of it
F16_MFMA_PEAK_TFLOPS = 2516.6
PEAK_BY_COMPUTE = {"f32": (F32_MFMA_PEAK_TFLOPS, "conv_encoder_kernel (10 MovementConvEncoders, exact f32 MFMA)"),
                   "f32x3": (F16_MFMA_PEAK_TFLOPS / 3, "conv_encoder_x3s_kernel (10 MovementConvEncoders, "
                                                      "3xfp16 split MFMA, staggered halves, peak = dense F16 MFMA / 3)"),
                   "f16": (F16_MFMA_PEAK_TFLOPS, "conv_encoder_f16w_kernel (10 MovementConvEncoders on 1..6-window "
                                                 "units, single fp16 MFMA per product, peak = dense F16 MFMA)")}
F16_X3S_KNAME = ("conv_encoder_x3s_kernel<false> (10 MovementConvEncoders, staggered halves, single fp16 MFMA per "
                 "product, peak = dense F16 MFMA)")


def f16_conv_is_x3s() -> bool:
    """The f16 mode's conv kernel, as vge_api.cpp picks it: the staggered x3s kernel in single fp16 unless
    VGE_F16_X3S=0 (conv_encoder_f16w_kernel) or the stem is split (VGE_F16_MIX bit 1)."""
    return os.environ.get("VGE_F16_X3S", "1") != "0" and not (int(os.environ.get("VGE_F16_MIX", "2")) & 1)


ARITH = {"f32": "f32 in, f32 accumulate (v_mfma_f32_16x16x4_f32)",
         "f32x3": "f32 operands as fp16 hi + fp16 residual lo (power-of-two scaled per row/window/column), 3 f16 "
                  "MFMAs per product (hi*hi + hi*lo + lo*hi), f32 accumulate",
         "f16": "MovementConvEncoders (85% of the FLOPs): operands rounded to fp16 (power-of-two scaled per "
                "row/window/column), 1 f16 MFMA per product, f32 accumulate, f32 GELU (one-exp2 erf, |err| < 5e-7) "
                "and GroupNorm epilogues; transformer: 3xfp16 split (VGE_F16 default)"}
HBM_PEAK_GBS = 8000.0
FEAT_BYTES_PER_WINDOW = 32 * (1024 + 207 + 9 + 10 + 120) * 4 + 32 * 2596 * 4   # read + write
# transformer_x3_kernel per 32-frame window: the token matrix (32 x 256 x 256) + 4 post-norm
# layers of 33 tokens: in_proj 256->768, out_proj 256->256, FFN 256->1024->256, attention QK^T + PV (8 heads of 32)
TX_FLOP_PER_WINDOW = 2 * 32 * 256 * 256 + 4 * (2 * 33 * (256 * 768 + 256 * 256 + 2 * 256 * 1024) + 2 * 2 * 33 * 33 * 256)
TX_WEIGHT_BYTES = 12.85e6   # split weights streamed from L2 into each window's workgroup (3.21 M weights x 4 B)
# fuse_kernel per window: the 10 encoder outputs read (f32) + the fused frame vectors written
FUSE_BYTES_PER_WINDOW = 10 * 32 * 256 * 4 + 32 * 256 * 4


def device_peaks() -> dict:
    """MFMA peaks of the visible GPU from rocminfo (CU count x max engine clock x MFMA FLOP/CU/clk):
    dense f16 4 SIMDs x 1024 FLOP/clk, exact f32 4 x 64.  Falls back to the MI355X_MICROARCH.md figures (256 CUs,
    2.4 GHz) when rocminfo is unavailable; `source` says which."""
    import re
    import subprocess
    try:
        txt = subprocess.run(["rocminfo"], capture_output=True, text=True, timeout=60).stdout
        for agent in txt.split("*******")[1:]:
            if re.search(r"Device Type:\s+GPU", agent) and "gfx950" in agent:
                cus = int(re.search(r"Compute Unit:\s+(\d+)", agent).group(1))
                mhz = int(re.search(r"Max Clock Freq\. \(MHz\):\s+(\d+)", agent).group(1))
                return {"f16": cus * 4 * 1024 * mhz * 1e6 / 1e12, "f32": cus * 4 * 64 * mhz * 1e6 / 1e12,
                        "source": f"rocminfo: {cus} CUs x {mhz} MHz"}
    except (OSError, subprocess.SubprocessError, AttributeError, ValueError):
        pass
    return {"f16": F16_MFMA_PEAK_TFLOPS, "f32": F32_MFMA_PEAK_TFLOPS,
            "source": "MI355X_MICROARCH.md (rocminfo unavailable): 256 CUs x 2400 MHz"}


def make_clips(seed, start, n, T, kp_len=None):
    from vge import synth
    clips = []
    for i in range(start, start + n):
        c = synth.make_clip(seed, i, T, kp_len)
        clips.append({"pose": c.pose, "global_orient": c.global_orient, "betas": c.betas, "vit": c.vit,
                      "keypoints": c.keypoints})
    return clips


def setup_dist():
    """One process per GPU (torchrun's env): rank r on GPU LOCAL_RANK over RCCL.  The world size reported in the line
    is the process group's (dist.get_world_size()), not the --gpus argument."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # one process per GPU over RCCL ("nccl").  VGE_BENCH_BACKEND=gloo rehearses the multi-rank code path
        # with ranks sharing the visible GPUs (a one-GPU box); the driver's scaling runs use the default.
        backend = os.environ.get("VGE_BENCH_BACKEND", "nccl")
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        world, rank = dist.get_world_size(), dist.get_rank()
    else:
        torch.cuda.set_device(0)
    return world, rank, torch.device("cuda", torch.cuda.current_device())


def gather_rank_times(dt: float, videos: int, world: int, dev) -> list:
    """[(seconds, videos)] of every rank in rank order (an all-gather over the bench's process group; RCCL takes
    device tensors, gloo host ones)."""
    if world == 1:
        return [(dt, videos)]
    on = dev if dist.get_backend() == "nccl" else "cpu"
    mine = torch.tensor([dt, float(videos)], dtype=torch.float64, device=on)
    got = [torch.empty_like(mine) for _ in range(dist.get_world_size())]
    dist.all_gather(got, mine)
    return [(float(g[0]), int(g[1])) for g in got]


def allreduce_sum(t, world):
    # vge.dist: one all-gather + rank-ordered sum (deterministic, identical on every rank)
    from vge.dist import allgather_sum
    return allgather_sum(t) if world > 1 else t


def cpu_share() -> int:
    """CPUs this process may use: the affinity mask, capped by a cgroup v2 quota (cpu.max) -- on the GPU box the
    affinity mask can count the whole machine while the job's share is 16 -- and by OMP_NUM_THREADS when set."""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, -(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


class _ClipWindows(torch.utils.data.Dataset):
    """The reference's WindowDataset role (utils.py:383-516) for the CPU baseline: the 32-frame windows of a clip
    (starts 0, 8, ...: one for config 2's 32-frame clips, five for config 5's 64-frame ones), featurised by the oracle
    in the DataLoader worker (clips are in memory: no npz decode, like the GPU leg)."""

    def __init__(self, clips, mean, std, starts=(0,)):
        self.clips, self.mean, self.std, self.starts = clips, mean, std, tuple(starts)

    def __len__(self):
        return len(self.clips)

    def __getitem__(self, i):
        from oracle.featurize import featurize_window
        c = self.clips[i]
        f = np.stack([featurize_window(c["pose"], c["global_orient"], c["betas"], c["vit"], c["keypoints"], s0, None)
                      for s0 in self.starts])
        return torch.from_numpy((f - self.mean) / (self.std + np.float32(1e-6))), i


def cpu_baseline(seconds: float, clips_per_batch: int = 32, workers: int = 4, T: int = CLIP_LEN):
    """Oracle CPU restatement of eval.py's generated-set pass in the reference's structure (eval.py:410-418,
    168-206): DataLoader(batch_size=32, num_workers=4) featurising in worker processes, the torch-fp32 encoder in
    the main process on this process's CPU share, then AC/TC (a clip's windows: its AC from their mean embedding, its
    TC the mean of their terms).  T: frames per clip (32: config 2, one window; 64: config 5, five).  Bounded: batches
    of 32 clips until `seconds` of wall time have elapsed.  Runs before the GPU is touched (the workers are forked)."""
    from oracle import evalflow
    from oracle.encoder import OracleEncoder
    from vge import synth
    share = cpu_share()
    torch.set_num_threads(share)
    sd = synth.make_state_dict(synth.DIMS_RAW, synth.DIMS_DIFF)
    enc = OracleEncoder(sd, synth.DIMS_RAW, synth.DIMS_DIFF)
    rng = np.random.default_rng(0)
    mean = rng.normal(0, 0.1, 2596).astype(np.float32)
    std = rng.uniform(0.5, 2.0, 2596).astype(np.float32)
    cents = torch.nn.functional.normalize(torch.randn(10, 256), dim=-1)
    label = {c: i for i, c in enumerate(evalflow.ACTION_CLASSES)}
    # a pool of clips generated up front (data synthesis is not part of the reference's work), passed over
    # repeatedly until `seconds` have elapsed
    n_clips = 1024 if T == CLIP_LEN else 512
    starts = list(range(0, T - CLIP_LEN + 1, 8))
    clips = make_clips(synth.SEED_GEN, 10_000, n_clips, T)
    names = [synth.generated_name(10_000 + i) + ".npz" for i in range(n_clips)]
    cls_all = [evalflow.ACTION_CLASSES[((10_000 + i) // 5) % 10] for i in range(n_clips)]
    loader = torch.utils.data.DataLoader(_ClipWindows(clips, mean, std, starts), batch_size=clips_per_batch,
                                         shuffle=False, num_workers=workers, multiprocessing_context="fork")
    n_done = 0
    marks = []  # (seconds, clips) after every batch: the spread over the sample's quarters is reported
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for feats, idx in loader:
            seq, fe, _ = enc.forward(feats.reshape(-1, *feats.shape[2:]))
            idx = [i for i in idx.tolist() for _ in starts]   # one name per window (eval.py groups by video)
            evalflow.ac_scores(seq, [cls_all[i] for i in idx], [names[i] for i in idx], cents, label)
            evalflow.tc_scores(fe, [names[i] for i in idx])
            n_done += len(idx) // len(starts)
            marks.append((time.perf_counter() - t0, n_done))
            if time.perf_counter() - t0 >= seconds:
                break
    t_used = time.perf_counter() - t0
    del loader
    quarters = []
    for q in range(4):  # videos/s within each quarter of the sample (the first one includes the worker start-up)
        lo, hi = q * t_used / 4, (q + 1) * t_used / 4
        seg = [(t, n) for t, n in marks if lo <= t <= hi]
        if len(seg) >= 2:
            quarters.append((seg[-1][1] - seg[0][1]) / max(seg[-1][0] - seg[0][0], 1e-9))
    return {"value": n_done / t_used, "unit": "videos/s", "cores": share, "kind": "port",
            "quarter_rates": [round(v, 1) for v in quarters],
            "sample": f"{n_done} synthetic {T}-frame clips ({len(starts)} window(s) each; in-memory features, no npz "
                      f"decode) through the reference's "
                      f"structure: DataLoader(batch_size={clips_per_batch}, num_workers={workers}) running the oracle "
                      f"featuriser (numpy) in worker processes, torch-fp32 oracle encoder on {share} threads (the "
                      f"process's CPU share) + AC/TC, {t_used:.1f} s wall"}


def oracle_precision(clips, mean, std, centroids, vcls, seq_gpu, ac_gpu, tc_gpu, starts=(0,), n: int = 64) -> dict:
    """|Δ| of the GPU step's outputs vs the oracle (CPU restatement of utils.py featurisation + model.py + eval.py
    metrics, pinned to the reference by tests/golden) on the first `n` clips of the timed workload, with the same
    stats and centroids.  Each clip has len(starts) windows: TC = float64 mean of the per-window terms
    (eval.py:209-226), AC = || normalize(mean_w seq_embed_w) - centroid || (eval.py:229-257)."""
    from oracle.encoder import OracleEncoder
    from oracle.featurize import featurize_window
    from vge import synth
    n, nw = min(n, len(clips)), len(starts)
    mean_h, std_h = mean.cpu().numpy(), std.cpu().numpy()
    feats = torch.from_numpy(np.stack([
        (featurize_window(c["pose"], c["global_orient"], c["betas"], c["vit"], c["keypoints"], s0, None) - mean_h)
        / (std_h + np.float32(1e-6)) for c in clips[:n] for s0 in starts]))
    sd = synth.make_state_dict(synth.DIMS_RAW, synth.DIMS_DIFF)
    seq, fe, _ = OracleEncoder(sd, synth.DIMS_RAW, synth.DIMS_DIFF).forward(feats)
    f = fe[:, 1:]
    tc = (f[:, 1:] - f[:, :-1]).norm(dim=-1).mean(dim=1).double().view(n, nw).mean(dim=1)
    cent = centroids.cpu()
    cls = vcls[:n].cpu().long()
    z = torch.nn.functional.normalize(seq.view(n, nw, -1).mean(dim=1), dim=-1)
    ac = (z - cent[cls]).norm(dim=-1)
    return {"vs": "oracle (CPU fp32 restatement of the reference, pinned by reference-generated golden vectors)",
            "clips": n, "windows": n * nw, "max_abs_ac": float((ac - ac_gpu[:n].cpu()).abs().max()),
            "max_abs_tc": float((tc - tc_gpu[:n].cpu()).abs().max()),
            "max_abs_seq_embed": float((seq - seq_gpu[: n * nw].cpu()).abs().max()), "north_star_tolerance": 1e-4}


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_command(args, env, argv, port=None):
    """The rank launch for `--gpus N`: None when this process is itself the (only) rank -- N = 1, or under torchrun
    (WORLD_SIZE set, which must then equal N) -- else the torch.distributed.run command that starts N ranks of this
    script on 127.0.0.1 (one process per GPU; the children see WORLD_SIZE and run the benchmark)."""
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if args.gpus is not None and int(ws) != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws} (torchrun --nproc-per-node)")
        return None
    if args.gpus is None or args.gpus <= 1:
        return None
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port if port is not None else _free_port()),
            str(Path(__file__).resolve()), *argv]


def launch_ranks(args, cmd) -> int:
    """Parent of a self-launched N-rank run: the CPU baseline first (this process never touches the GPU: it
    is measured on the host before any rank starts, and handed to rank 0 in the environment), then torchrun as a
    CHILD process (never exec: nothing here has initialised the GPU, but the ranks must be fresh processes anyway);
    rank 0's JSON line goes straight to this process's stdout.  Returns the children's exit status."""
    import subprocess
    env = dict(os.environ)
    if args.workload in ("score", "tag", "cfg5") and not args.no_cpu_baseline:
        if args.workload == "score":
            cpu = cpu_baseline(args.cpu_seconds)
        elif args.workload == "cfg5":
            cpu = cpu_baseline(args.cpu_seconds, T=64)
        else:
            import bench_tag
            cpu = (bench_tag.cpu_baseline_extract(args.cpu_seconds) if getattr(args, "extract", False)
                   else bench_tag.cpu_baseline())
        env["VGE_BENCH_CPU_BASELINE"] = json.dumps(cpu)
    env.setdefault("OMP_NUM_THREADS", str(max(1, cpu_share() // args.gpus)))
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of this node.  Without torchrun's WORLD_SIZE and N > 1, bench.py launches N ranks "
                         "itself (torch.distributed.run as a child process, before any GPU call); under torchrun it "
                         "must equal WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--clips", type=int, default=256, help="32-frame clips per GPU per step (config 2: 256)")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--compute", default=None, choices=["f32x3", "f32", "f16"],
                    help="f32x3: 3xfp16 split-precision MFMA (f32-class, default of score/tag/e2e); f32: exact f32 "
                         "MFMA; f16: single-fp16 MFMA throughput mode (default of cfg5)")
    ap.add_argument("--chunk", type=int, default=4096, help="cfg5: windows per featurise + encode launch")
    ap.add_argument("--chunk-clips", type=int, default=32, help="e2e: clips per extraction pass (frames in HBM)")
    ap.add_argument("--no-throughput-mode", action="store_true",
                    help="score: skip the second (f16) run reported as throughput_mode beside the f32x3 headline")
    ap.add_argument("--pipeline", default=None, choices=["side3", "side2", "side", "tail", "serial"],
                    help="score/cfg5 stream layout: side = the next chunk is featurised on a second stream beside the "
                         "current chunk's fusion + transformer; side2 = side, plus the per-video scores and "
                         "their host copies on that second stream (two output buffers, alternate steps); tail = the "
                         "transformer / outputs / scores run on a second stream (vge_encoder_set_tail_stream) while "
                         "the encode stream featurises the next chunk and queues its conv stage, which then takes CUs "
                         "as the transformer's workgroups finish (its hipEvents include that wait, so the conv "
                         "roofline is not measured in this mode); serial = one stream, featurise right before each "
                         "encode (default); side3 = side2 with each step's scores launched on the side stream after "
                         "the NEXT step's conv (which follows this step's transformer on the encode stream), ahead of "
                         "its featurise, so no marker follows the transformer (measured +0.9-1.1 %% videos/s, same "
                         "box); the last step's scores are launched after the loop, inside the timed region.  "
                         "Default: serial (score: the overlapped featurise slows the transformer by about its own "
                         "time, 185.0k-185.4k vs 183.3k-185.0k videos/s for side3, same box, round 5; cfg5: its "
                         "occupancy-2 fp16 transformer fills every register of a CU, so an overlapped featurise only "
                         "waits for its workgroups)")
    ap.add_argument("--serial-featurize", action="store_true", help="= --pipeline serial")
    ap.add_argument("--host-scores", default="direct", choices=["direct", "copy"],
                    help="score/cfg5: the per-video AC / TC reach pinned host memory written by the score kernel itself "
                         "(direct, default: no copy kernels in the step) or through two device-to-host copies (copy)")
    ap.add_argument("--event-every", type=int, default=5,
                    help="record the conv stage's (and featurise's) hipEvents on every k-th timed step, from the first: "
                         "each event is a queue marker (measured: all steps 184.2k-185.4k videos/s, every 5th "
                         "186.4k-186.5k, same box)")
    ap.add_argument("--serial-extract", action="store_true",
                    help="e2e: run TokenHMR and DWPose one after the other on one stream (default: two streams)")
    ap.add_argument("--no-detector", action="store_true",
                    help="e2e: skip DWPose's YOLOX person detector (every frame takes the whole-frame pose box)")
    ap.add_argument("--extract", action="store_true",
                    help="tag: config 4 end to end -- each rank extracts its shard of the generated videos from frames "
                         "(gate detector + TokenHMR, YOLOX-L + DWPose -> npz / keypoints.npy) before the sharded flow "
                         "(bench_tag.run_extract)")
    ap.add_argument("--no-e2e", action="store_true",
                    help="score at N = 1: skip the nested `e2e` record (config 3, run as a child process after the "
                         "config-2 line's measurements)")
    ap.add_argument("--e2e-clips", type=int, default=1000, help="clips of the nested config-3 record (config 3: 1k)")
    ap.add_argument("--e2e-timeout", type=float, default=420.0, help="seconds the nested config-3 child may take")
    ap.add_argument("--workload", default="score", choices=["score", "e2e", "tag", "cfg5"],
                    help="score: config 2 (default, the bench line); e2e: config 3, frames -> TokenHMR + DWPose -> "
                         "scores (bench_e2e.py; --clips defaults to 8 there); tag: config 4 on pre-extracted "
                         "features, the full sharded eval flow over 300 videos (bench_tag.py); cfg5: config 5, --clips "
                         "(default 10000) 64-frame clips sharded over the ranks, f16 MFMA path by default")
    args = ap.parse_args()
    cmd = launch_command(args, os.environ, sys.argv[1:])
    if cmd is not None:
        sys.exit(launch_ranks(args, cmd))
    if args.compute is None:
        args.compute = "f16" if args.workload == "cfg5" else "f32x3"
    if args.workload == "cfg5" and args.compute == "f16":
        # config 5 is the throughput-ceiling run of "the fp16 MFMA path": the transformer in fp16 too (its
        # precision is still measured against the oracle and reported)
        os.environ.setdefault("VGE_F16_MIX", "0")
    if args.workload == "cfg5" and args.clips == 256:
        args.clips = 10_000
    if args.pipeline is None:
        args.pipeline = "serial"

    cpu = json.loads(os.environ["VGE_BENCH_CPU_BASELINE"]) if os.environ.get("VGE_BENCH_CPU_BASELINE") else None
    if cpu is None and args.workload in ("score", "cfg5") and int(os.environ.get("WORLD_SIZE", "1")) == 1 and \
            not args.no_cpu_baseline:
        # before the GPU is initialised: its DataLoader workers are forked
        cpu = cpu_baseline(args.cpu_seconds, T=64 if args.workload == "cfg5" else CLIP_LEN)
    if cpu is None and args.workload == "tag" and int(os.environ.get("WORLD_SIZE", "1")) == 1 and \
            not args.no_cpu_baseline:
        import bench_tag
        cpu = bench_tag.cpu_baseline_extract(args.cpu_seconds) if args.extract else bench_tag.cpu_baseline()
    world, rank, dev = setup_dist()
    if args.workload == "tag":
        import bench_tag
        out = (bench_tag.run_extract if args.extract else bench_tag.run)(args, world, rank, dev, METRIC, cpu)
        if rank == 0:
            print(json.dumps(out))
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    if args.workload == "e2e":
        import bench_e2e
        if args.clips == 256:
            args.clips = 8
        out = bench_e2e.run(args, world, rank, dev, METRIC, allreduce_sum, make_clips)
        if rank == 0:
            print(json.dumps(out))
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return
    out = run_score(args, world, rank, dev)
    if args.workload == "score" and args.compute == "f32x3" and not args.no_throughput_mode:
        # the fp16-operand throughput mode on the same workload, reported nested beside the f32-class headline
        import copy
        pa = copy.copy(args)
        pa.compute, pa.steps, pa.warmup = "f16", max(5, args.steps // 2), 2
        thr = run_score(pa, world, rank, dev)
        if rank == 0:
            out["throughput_mode"] = {k: thr[k] for k in ("dtype", "value", "ms_per_step", "steps", "precision",
                                                          "roofline", "stage_ms")}
    if rank == 0:
        out["cpu_baseline"] = cpu
        if args.workload == "score" and world == 1 and not args.no_e2e:
            out["e2e"] = run_e2e_child(args)
        print(json.dumps(out))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def run_e2e_child(args) -> dict:
    """BASELINE config 3 -- the north star's "videos/sec on synthetic 32-frame 256x256 clips": frames in HBM -> the
    Faster R-CNN gate + TokenHMR and YOLOX + DWPose extractors -> featurise -> encoder -> AC/TC (bench_e2e.py;
    reference path eval.py:350-466 fed by extract_mesh.py:150-241 / process_video.py:59-94), `--e2e-clips` clips, 1
    timed step after 1 warm-up, with its own stage_ms, rooflines (ViT-H GEMMs, the gate detector), PMC traffic and CPU
    baseline.  Run as a child process (never exec) after this line's measurements, so its ~40 GB of frames and
    extractor workspaces do not share the config-2 timing; its heartbeat lines go to stderr.  A failure or timeout is
    recorded in the returned dict; the config-2 line is printed either way."""
    import subprocess
    cmd = [sys.executable, str(Path(__file__).resolve()), "--workload", "e2e", "--clips", str(args.e2e_clips),
           "--steps", "1", "--warmup", "1", "--cpu-seconds", "15"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    t0 = time.perf_counter()
    print("[bench] config-2 line measured; the nested config-3 run starts", file=sys.stderr, flush=True)
    try:
        r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=None, text=True, timeout=args.e2e_timeout)
    except subprocess.TimeoutExpired:
        return {"error": f"timed out after {args.e2e_timeout:.0f} s", "cmd": " ".join(cmd[1:])}
    wall = time.perf_counter() - t0
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"exit status {r.returncode}", "cmd": " ".join(cmd[1:]), "stdout_tail": r.stdout[-2000:]}
    e = json.loads(lines[-1])
    e["child_wall_s"] = wall
    e["cmd"] = " ".join(cmd[1:])
    return e


def tx_peak(compute: str, pk: dict) -> float:
    """The transformer's MFMA ceiling: it runs the 3xfp16 split in f32x3 and, by default, in f16 (VGE_F16_MIX bit 2);
    activations-only split (bit 4): 2 MFMAs per product; VGE_F16_MIX=0: single fp16; exact f32 in f32."""
    if compute == "f32":
        return pk["f32"]
    if compute == "f32x3":
        return pk["f16"] / 3
    mix = int(os.environ.get("VGE_F16_MIX", "2"))
    return pk["f16"] / 3 if mix & 2 else (pk["f16"] / 2 if mix & 4 else pk["f16"])


def stage_roofline(stage_ms: dict, feat_ms: float, score_ms: float, windows_per_encode: int, windows_per_step: int,
                   videos: int, mfma_peak: float, tx_mfma_peak: float, steps: int, dt: float) -> dict:
    """Every hot kernel of the step against its ceiling, from the same hipEvents as `stage_ms` (conv: the timed steps;
    the others: the untimed steps after them).  MFMA kernels in algorithmic TFLOP/s against the compute mode's MFMA
    ceiling; HBM kernels in algorithmic GB/s against HBM peak; the transformer also as its L2->CU weight stream (one
    full image per window).  `whole_path`: the encoder's 2.0203 GFLOP per window at the measured windows/s."""
    def mfma(flop, ms, peak=mfma_peak):
        a = flop / (ms * 1e-3) / 1e12 if ms > 0 else None
        return {"bound": "mfma", "achieved": a, "peak": peak, "unit": "TFLOP/s", "frac": a / peak if a else None,
                "flop_per_launch": flop, "avg_launch_ms": ms}

    def hbm(nbytes, ms):
        a = nbytes / (ms * 1e-3) / 1e9 if ms > 0 else None
        return {"bound": "hbm", "achieved": a, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": a / HBM_PEAK_GBS if a else None,
                "bytes_per_launch": nbytes, "avg_launch_ms": ms}

    W = windows_per_encode
    tx = mfma(TX_FLOP_PER_WINDOW * W, stage_ms.get("transformer", 0.0), tx_mfma_peak)
    tx["l2_weight_stream_GBs"] = TX_WEIGHT_BYTES * W / (tx["avg_launch_ms"] * 1e-3) / 1e9 if tx["avg_launch_ms"] else None
    tx["traffic"] = pmc_kernel_traffic("transformer_x3_kernel", W)
    whole = ENCODER_FLOP_PER_WINDOW * windows_per_step * steps / dt / 1e12
    fuse = hbm(FUSE_BYTES_PER_WINDOW * W, stage_ms.get("fusion_pool", 0.0))
    fuse["traffic"] = pmc_kernel_traffic("fuse_kernel", W)
    feat = hbm(FEAT_BYTES_PER_WINDOW * W, feat_ms)
    feat["traffic"] = pmc_kernel_traffic("featurize_tiles_kernel", W)
    # score_videos: per window its seq embedding + TC term, per video its centroid and two outputs
    score = hbm(windows_per_step * (256 + 1) * 4 + videos * (256 * 4 + 4 + 8 + 4), score_ms)
    score["traffic"] = pmc_kernel_traffic("score_videos_kernel", windows_per_step)
    return {
        "conv_encoders": mfma(CONV_FLOP_PER_WINDOW * W, stage_ms.get("conv_encoders", 0.0)),
        "transformer": tx,
        "fusion_pool": fuse,
        "featurize": feat,
        "score_videos": score,
        "whole_path": {"achieved": whole, "peak": mfma_peak, "unit": "TFLOP/s", "frac": whole / mfma_peak,
                       "flop_per_window": ENCODER_FLOP_PER_WINDOW},
        "traffic_source": "profiles/pmc_kernels.json (tools/pmc_kernels.py; null where the pass predates the kernel's "
                          "sources)",
    }


# the sources each measured kernel is compiled from: a committed PMC pass counts for a kernel only while these are
# unchanged (its `source_sha`)
KERNEL_SOURCES = {
    "conv_encoders": ("vge_encoder_x3.hip", "vge_encoder_x3s.hip", "vge_x3.h", "vge_common.h"),
    "transformer_x3_kernel": ("vge_transformer_x3.hip", "vge_x3.h", "vge_common.h"),
    "featurize_tiles_kernel": ("vge_featurize.hip", "vge_common.h"),
    "fuse_kernel": ("vge_encoder.hip", "vge_common.h"),
    "score_videos_kernel": ("vge_score.hip", "vge_common.h"),
}


def sources_sha(files) -> str:
    import hashlib
    h = hashlib.sha256()
    for f in files:
        h.update((ROOT / "video-gen-evals_amd" / "csrc" / f).read_bytes())
    return h.hexdigest()[:16]


def _kernel_sources_sha() -> str:
    return sources_sha(KERNEL_SOURCES["conv_encoders"])


def pmc_kernel_traffic(kernel: str, windows: int):
    """HBM bytes per launch of one of the step's other kernels from the committed PMC pass (profiles/pmc_kernels.json,
    tools/pmc_kernels.py: FETCH_SIZE x 2 + WRITE_SIZE), scaled to `windows`, only if taken on this tree's sources."""
    try:
        e = json.loads((ROOT / "profiles" / "pmc_kernels.json").read_text())[kernel]
        if e.get("source_sha") != sources_sha(KERNEL_SOURCES[kernel]):
            return None
        return e["hbm_bytes_per_launch"] / e["windows_per_launch"] * windows
    except (OSError, KeyError, ValueError, ZeroDivisionError):
        return None


def pmc_traffic(compute: str, windows: int):
    """HBM bytes per launch of the conv kernel from the committed PMC pass (profiles/pmc_conv_encoder.json:
    FETCH_SIZE x 2 + WRITE_SIZE per the microarchitecture guide), only if that pass was taken on the kernel sources
    of this tree (source hash recorded in the file); otherwise None."""
    pmc = ROOT / "profiles" / "pmc_conv_encoder.json"
    try:
        pj = json.loads(pmc.read_text())
        e = pj[compute]
        if e.get("source_sha") != _kernel_sources_sha():
            return None
        if compute == "f16" and e.get("kernel") != ("conv_encoder_x3s_kernel" if f16_conv_is_x3s()
                                                     else "conv_encoder_f16w_kernel"):
            return None
        return e["hbm_bytes_per_window"] * windows
    except (OSError, KeyError, ValueError):
        return None


def run_score(args, world, rank, dev):
    """config 2 (`score`: 256 clips x 32 frames per GPU, one window each, weak scaling) and config 5 (`cfg5`:
    10k clips x 64 frames = 5 windows each, sharded over the ranks, strong scaling).  One step = featurise every
    window -> encode (in chunks of `--chunk` windows) -> per-video AC + TC -> scores to pinned host memory."""
    from vge import eval as VE
    from vge import ops, synth
    from vge.data import ACTION_CLASSES, pack_frame_store
    from vge.dist import shard, shard_bounds
    cfg5 = args.workload == "cfg5"
    T = 64 if cfg5 else CLIP_LEN
    starts = list(range(0, T - CLIP_LEN + 1, 8))
    if cfg5:
        lo, hi = shard_bounds(args.clips, rank, world)
    else:
        lo, hi = rank * args.clips, (rank + 1) * args.clips
    V = hi - lo
    NW = V * len(starts)
    CH = min(NW, args.chunk) if cfg5 else NW

    # ---------------- setup: frame stores in HBM, stats + centroids over the (sharded) real set
    t_setup = time.perf_counter()
    n_real_per_class, T_real = 8, 64
    real_idx = shard(list(range(10 * n_real_per_class)), rank, world)     # contiguous block of the real set
    real_clips = [make_clips(synth.SEED_REAL, i, 1, T_real)[0] for i in real_idx]
    real_cls = [ACTION_CLASSES[i // n_real_per_class] for i in real_idx]
    real_store = ops.DeviceFrameStore.from_host(pack_frame_store(real_clips, [f"r{i}" for i in real_idx], real_cls), dev)
    sums = torch.zeros((2, ops.FEAT_DIM), device=dev, dtype=torch.float64)
    counts = np.zeros(2, np.int64)
    ops.stats_accumulate(real_store, range(real_store.n_videos), sums, counts)
    sums = allreduce_sum(sums, world)
    counts = allreduce_sum(torch.tensor(counts, device=dev), world).cpu().numpy()
    mean, std = ops.stats_finalize(sums, counts)
    stats = VE.ModalityStatsGPU(mean, std, sums, counts)
    sd = synth.make_state_dict(synth.DIMS_RAW, synth.DIMS_DIFF)
    enc = ops.Encoder(sd, device=dev, compute=args.compute)
    enc.reserve(max(CH, 64))
    real_win = torch.tensor([[v, s] for v in range(real_store.n_videos) for s in range(0, T_real - CLIP_LEN + 1, 8)],
                            dtype=torch.int32, device=dev)
    rseq, _, _ = VE.encode_windows(enc, real_store, real_win, stats, batch=max(CH, 64))
    label = {c: i for i, c in enumerate(ACTION_CLASSES)}
    y = torch.tensor([label[real_cls[v]] for v in range(real_store.n_videos) for _ in range(0, T_real - CLIP_LEN + 1, 8)],
                     dtype=torch.int32, device=dev)
    csum = torch.zeros((10, 256), device=dev)
    ccnt = torch.zeros((10,), device=dev)
    ops.centroid_accumulate(rseq, y, csum, ccnt)
    centroids = ops.centroid_finalize(allreduce_sum(csum, world), allreduce_sum(ccnt, world))

    if cfg5:  # 10k clips: generated on host threads (numpy's generators release the GIL)
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max_workers=cpu_share()) as ex:
            gen_clips = list(ex.map(lambda k: make_clips(synth.SEED_GEN, k, 1, T)[0], range(lo, hi)))
    else:
        gen_clips = make_clips(synth.SEED_GEN, lo, V, T)
    names = [synth.generated_name(k) for k in range(lo, hi)]
    gstore = ops.DeviceFrameStore.from_host(pack_frame_store(gen_clips, names, ["X"] * V), dev)
    windows = torch.tensor([[v, s0] for v in range(V) for s0 in starts], dtype=torch.int32, device=dev)
    first = torch.arange(0, NW + 1, len(starts), dtype=torch.int32, device=dev)
    vcls = torch.tensor([label[ACTION_CLASSES[(k // 5) % 10]] for k in range(lo, hi)], dtype=torch.int32, device=dev)
    feats = torch.empty((CH, CLIP_LEN, ops.FEAT_DIM), device=dev)
    seq = torch.empty((NW, 256), device=dev)
    tcw = torch.empty((NW,), device=dev)
    # side2: scores run on the side stream while the next step's encodes write the other buffer pair
    seq_b, tcw_b = [seq, torch.empty_like(seq)], [tcw, torch.empty_like(tcw)]
    n_step = [0]
    n_timed = [0]  # timed steps started (the --event-every sampling)
    host_ac = torch.empty((V,), dtype=torch.float32, pin_memory=True)
    host_tc = torch.empty((V,), dtype=torch.float64, pin_memory=True)
    n_chunks = (NW + CH - 1) // CH
    fe0 = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps * n_chunks + 1)]
    fe1 = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps * n_chunks + 1)]
    n_fe = [0]  # featurise launches timed so far (inside the timed steps)
    timing = [False]
    side = torch.cuda.Stream(device=dev)
    feat_ready = torch.cuda.Event()
    pending = [None]  # the chunk whose featurise is already enqueued on `side`

    def featurize_chunk(c, stream):
        b0, b1 = c * CH, min(NW, (c + 1) * CH)
        # (its events follow the conv's sampling: every --event-every-th timed step)
        k = n_fe[0] if timing[0] and n_timed[0] % args.event_every == 0 else None
        if k is not None:
            fe0[k].record(stream)
        ops.featurize(gstore, windows[b0:b1], stats.mean, stats.std, out=feats[: b1 - b0])
        if k is not None:
            fe1[k].record(stream)
            n_fe[0] += 1

    deferred = [None]  # side3: (seq, tc) buffers of the step whose scores are not launched yet

    def scores_to_host(sq, tw):
        """per-video AC / TC into the pinned host buffers: written by the score kernel itself (--host-scores direct,
        the default) or computed on the device and copied (copy: two blit kernels after it)"""
        if args.host_scores == "direct":
            return ops.score_videos(sq, tw, first, vcls, centroids, out=(host_ac, host_tc))
        ac, tc = ops.score_videos(sq, tw, first, vcls, centroids)
        host_ac.copy_(ac, non_blocking=True)
        host_tc.copy_(tc, non_blocking=True)
        return ac, tc

    def launch_scores(stream, sq, tw):
        with torch.cuda.stream(stream):
            return scores_to_host(sq, tw)

    def launch_feat(c):
        # featurise chunk c on the side stream once the last encode's conv stage (the last reader of feats) is done:
        # it runs beside that chunk's fusion + transformer, on the CUs the transformer's workgroups leave free
        # (every featurise workgroup reserves its kernel's static LDS, ~46 KB, which does not fit beside a transformer
        # workgroup's 139 KB: the two share the chip, not a CU)
        with torch.cuda.stream(side):
            enc.wait_conv(side)
            if deferred[0] is not None:
                # side3: the previous step's scores -- its transformer ran before this conv on the encode stream --
                # ahead of this featurise (same box: 188.4k-188.8k videos/s this way, 187.8k-188.0k behind it), whose
                # feat_ready gates the conv (and so the transformer) that next rewrites their buffer pair
                launch_scores(side, *deferred[0])
                deferred[0] = None
            featurize_chunk(c, side)
            feat_ready.record(side)
        pending[0] = c

    mode = "serial" if args.serial_featurize else args.pipeline
    tail = torch.cuda.Stream(device=dev) if mode == "tail" else None
    enc.set_tail_stream(tail)
    tx_done = torch.cuda.Event()

    sc_ev = []  # (start, end) events around standalone per-video score launches after the timed steps

    def drain():
        """side3: launch the deferred scores now (after the last transformer: one marker)"""
        if deferred[0] is None:
            return None, None
        cur = torch.cuda.current_stream()
        tx_done.record(cur)
        side.wait_event(tx_done)
        out = launch_scores(side, *deferred[0])
        deferred[0] = None
        return out

    def step(i=None, flush=False):
        ac = tc = None
        cur = torch.cuda.current_stream()
        sq, tw = (seq_b[n_step[0] % 2], tcw_b[n_step[0] % 2]) if mode in ("side2", "side3") else (seq, tcw)
        n_step[0] += 1
        for c in range(n_chunks):
            b0, b1 = c * CH, min(NW, (c + 1) * CH)
            if mode == "serial" or (mode == "tail" and pending[0] != c):
                featurize_chunk(c, cur)
            elif mode in ("side", "side2", "side3"):
                if pending[0] != c:
                    launch_feat(c)
                cur.wait_event(feat_ready)
            if timing[0]:  # the conv stage's two events on every --event-every-th step of the timed region
                enc.profile_mask(0x3 if n_timed[0] % args.event_every == 0 else 0)
            enc.encode(feats[: b1 - b0], frame_embed=False, tc=True, seq_out=sq[b0:b1], tc_out=tw[b0:b1])
            if mode in ("side", "side2", "side3"):
                launch_feat((c + 1) % n_chunks)  # the next chunk, or the next step's first
            if mode == "tail":
                # the next chunk (or the next step's first) on the encode stream, beside this chunk's transformer
                # on the tail stream; the next encode's conv stage follows it there
                featurize_chunk((c + 1) % n_chunks, cur)
                pending[0] = (c + 1) % n_chunks
        if mode == "side3":
            deferred[0] = (sq, tw)
            return drain() if flush else (None, None)
        if mode == "side2":
            # after the last transformer, on the side stream behind the next step's first featurise: the next conv
            # waits for that featurise (feat_ready), not for the scores; the step after next rewrites this buffer
            # pair only after a later featurise on the same side stream, so after these scores
            tx_done.record(cur)
            side.wait_event(tx_done)
        sst = tail if tail is not None else (side if mode == "side2" else cur)
        with torch.cuda.stream(sst):
            ac, tc = scores_to_host(sq, tw)
        return ac, tc

    # precision evidence for the timed mode: the untimed first step's scores vs the oracle on a sample of clips
    ac_a, tc_a = step(flush=True)
    torch.cuda.synchronize()  # the scores may come from the tail stream
    ac_a, tc_a = ac_a.clone(), tc_a.clone()  # (--host-scores direct: the pinned buffers every step rewrites)
    precision = oracle_precision(gen_clips, stats.mean, stats.std, centroids, vcls, seq, ac_a, tc_a, starts,
                                 n=16 if cfg5 else V) if rank == 0 else None
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t_setup

    for k in range(args.warmup):
        step(flush=k == args.warmup - 1)  # (side3: no deferred scores carried into the timed steps)
    torch.cuda.synchronize()
    # inside the timed steps only the conv stage's two events are recorded (each event is a queue marker: all six
    # stage markers measured -1.3 % videos/s); the other stages are timed on untimed steps afterwards
    enc.profile_mask(0x3)
    enc.profile_begin(args.steps * n_chunks)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    timing[0] = True
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i, flush=i == args.steps - 1)  # side3: the last step's scores inside the timed region
        n_timed[0] += 1
    torch.cuda.synchronize()
    timing[0] = False
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    enc.status()  # the device status word of every timed launch (a host read after the synchronize above)
    enc.profile_mask(0x3)  # (profile_read finds the last recorded event from the mask)
    # every rank's (wall time, videos): the line's time is the max over ranks, `value` all ranks' videos / that time
    per_rank = gather_rank_times(dt, V, world, dev)
    dt = max(t for t, _ in per_rank)
    stage_ms, ncalls = enc.profile_read()
    n_extra = 5
    enc.profile_mask(0x3F)
    enc.profile_begin(n_extra * n_chunks)
    for k in range(n_extra):
        step(flush=k == n_extra - 1)
    torch.cuda.synchronize()
    # the per-video score kernel alone (in the pipelined step it runs on the side stream, where its events would also
    # span the next conv that holds every CU): 10 launches on the current stream, hipEvents around each
    sq_last, tw_last = (seq_b[(n_step[0] - 1) % 2], tcw_b[(n_step[0] - 1) % 2]) if mode in ("side2", "side3") else (seq, tcw)
    for _ in range(10):
        sc_ev.append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
        sc_ev[-1][0].record()
        ops.score_videos(sq_last, tw_last, first, vcls, centroids)
        sc_ev[-1][1].record()
    # featurise alone, likewise (in the pipelined step it shares the CUs with the transformer): 10 launches of the
    # first chunk on the current stream
    fs_ev = []
    b1 = min(NW, CH)
    for _ in range(10):
        fs_ev.append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
        fs_ev[-1][0].record()
        ops.featurize(gstore, windows[:b1], stats.mean, stats.std, out=feats[:b1])
        fs_ev[-1][1].record()
    torch.cuda.synchronize()
    score_ms = sum(a.elapsed_time(b) for a, b in sc_ev) / max(1, len(sc_ev))
    feat_alone_ms = sum(a.elapsed_time(b) for a, b in fs_ev) / max(1, len(fs_ev))
    stage_x, ncalls_x = enc.profile_read()
    stage_out = {k: (v / max(ncalls, 1) if k == "conv_encoders" else stage_x[k] / max(ncalls_x, 1))
                 for k, v in stage_ms.items()}
    feat_ms = sum(fe0[k].elapsed_time(fe1[k]) for k in range(n_fe[0])) / max(1, n_fe[0])
    assert np.isfinite(host_ac.numpy()).all() and np.isfinite(host_tc.numpy()).all()
    # every step scores the same windows: the last step's host copies (after the extra steps, which alternate the
    # side2 output buffers like the timed ones) must equal the first step's scores bit for bit
    last_equals_first = bool(np.array_equal(host_ac.numpy(), ac_a.cpu().numpy()) and
                             np.array_equal(host_tc.numpy(), tc_a.cpu().numpy()))
    if not last_equals_first:
        raise RuntimeError("bench: the last step's scores differ from the first step's")
    if rank != 0:
        return None
    conv_ms = stage_ms["conv_encoders"] / max(ncalls, 1)
    achieved = CONV_FLOP_PER_WINDOW * CH / (conv_ms * 1e-3) / 1e12
    _, kname = PEAK_BY_COMPUTE[args.compute]
    if args.compute == "f16" and f16_conv_is_x3s():
        kname = F16_X3S_KNAME
    pk = device_peaks()
    peak = {"f16": pk["f16"], "f32x3": pk["f16"] / 3, "f32": pk["f32"]}[args.compute]
    total_videos = sum(v for _, v in per_rank) * args.steps
    if cfg5:
        workload = (f"BASELINE config 5: {args.clips} synthetic 64-frame clips (5 windows each) sharded over "
                    f"{world} GPU(s), fusion-encoder fwd + AC/TC, pre-extracted features resident in HBM, "
                    f"{args.compute} MFMA path")
    else:
        workload = ("BASELINE config 2: fusion-encoder fwd + AC/TC metrics, 256 clips x 32 frames per GPU, "
                    "pre-extracted features resident in HBM (featurise included in the step)")
    return {
        "metric": METRIC,
        "value": total_videos / dt,
        "unit": "videos/s",
        "n_gpus": world,
        "ranks_seen": len(per_rank),
        "per_rank_videos_per_s": [v * args.steps / t for t, v in per_rank],
        "backend": dist.get_backend() if dist.is_initialized() else None,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if cfg5 else "weak",
        "vs_baseline": None,
        "dtype": args.compute,
        "precision": {"arith": ARITH[args.compute] if not (args.compute == "f16" and
                                                             os.environ.get("VGE_F16_MIX", "2") == "0") else
                      ARITH["f16"].replace("transformer: 3xfp16 split (VGE_F16 default)",
                                           "transformer: fp16 too (VGE_F16_MIX=0)"), **precision,
                      "last_step_equals_first": last_equals_first},
        "data": "synthetic (deterministic generator vge.synth: quaternion-walk SMPL rotations, N(0,1) betas/tokens, "
                "U[0,1] keypoints with 5% invisible; random-init weights of the reference architecture)",
        "config": {"workload": workload, "clips_per_gpu": V, "frames_per_clip": T, "windows_per_step_per_gpu": NW,
                   "windows_per_encode": CH, "parallelism": f"video-sharded x{world}"},
        "roofline": {"bound": "mfma", "kernel": kname,
                     "achieved": achieved, "peak": peak, "peak_source": pk["source"], "unit": "TFLOP/s",
                     "frac": achieved / peak, "traffic": pmc_traffic(args.compute, CH),
                     "flop_per_launch": CONV_FLOP_PER_WINDOW * CH, "avg_launch_ms": conv_ms},
        "stage_ms": stage_out,
        "stage_roofline": stage_roofline(stage_out, feat_ms, score_ms, CH, NW, V, peak, tx_peak(args.compute, pk),
                                         args.steps, dt),
        "stage_ms_source": "conv_encoders: hipEvents in the timed steps; the other stages: 5 untimed steps after them; "
                           "score_videos: 10 standalone launches after those",
        "featurize": {"avg_ms": feat_ms, "bound": "hbm", "overlapped": mode != "serial", "pipeline": mode,
                      "achieved_GBs": FEAT_BYTES_PER_WINDOW * CH / (feat_ms * 1e-3) / 1e9, "peak_GBs": HBM_PEAK_GBS,
                      "standalone": {"avg_ms": feat_alone_ms, "windows": b1,
                                     "achieved_GBs": FEAT_BYTES_PER_WINDOW * b1 / (feat_alone_ms * 1e-3) / 1e9,
                                     "source": "10 launches on the current stream after the timed steps, hipEvents"}},
        "encoder_tflops_2.0203GF_per_window": ENCODER_FLOP_PER_WINDOW * NW * args.steps / dt / 1e12,
        "setup_s": setup_s,
    }

if __name__ == "__main__":
    main()
