"""End-to-end workload of bench.py (`--workload e2e`, BASELINE.json configs[2]): 256x256 RGB frames resident in HBM
-> TokenHMR extractor (ViT-H/16 backbone + SMPL token-decoder head, bf16 MFMA; vge_hmr.h) and DWPose keypoints
(RTMPose-l whole-body, bf16 MFMA implicit-GEMM convs; vge_dwpose.h) writing the frame store -> featurise ->
fusion encoder (f32x3) -> AC/TC, per step `--clips` 32-frame clips per GPU.

The reference pipeline is extract_mesh.py (TokenHMR per frame, modifications/mesh_generator.py:119-171) + DWPose
(modifications/process_video.py) -> npz / keypoints.npy on disk -> eval.py.  Here the frames-to-scores path stays
in HBM and both extractors start from the full frames.  One YOLOX-L person detection per frame (640x640 letterbox)
serves both: DWPose runs as the reference's Wholebody does (RTMPose-l on persons 0 / 1, the whole frame when nobody
is found -> keypoints.npy rows), and TokenHMR's front end (mesh_generator.py:101-145; YOLOX-L stands in for its
detectron2 Faster R-CNN, absent offline) applies the single-person gate (exactly one person > 0.5) and crops every
frame with ViTDetDataset's warp (vge_hmr_crop).  The gate's decision is computed and reported (`front_end`); a frame
it rejects is still cropped (whole-frame box) and extracted, so the timed work is the every-frame-valid upper bound
whatever the random-weight detector finds.  `--no-detector`: whole-frame boxes for both extractors.  Parity for the
upstream models is unpinned.

Roofline: the backbone GEMM kernel (gemm_bf16_kernel, MFMA bound): achieved = algorithmic FLOPs of every backbone
GEMM launch / their summed durations (hipEvents recorded around each launch on the extract stream inside the timed
steps); peak = dense bf16 MFMA 2516.6 TFLOP/s.  cpu_baseline = oracle/hmr.py (the fp32 torch restatement of the
same ViT-H + head) + the scoring restatement on this host, bounded sample.
"""
from __future__ import annotations

import json
import os
import time

import numpy as np
import torch
import torch.distributed as dist

BF16_MFMA_PEAK_TFLOPS = 2516.6


def cpu_baseline_e2e(seconds: float, detector: bool = True):
    from oracle.dwpose import OracleRtmpose
    from oracle.hmr import OracleHmr
    from oracle.yolox import OracleYolox
    from vge import synth
    from vge.dwpose import RTMPOSE_L, YOLOX_L
    from vge.hmr import TOKENHMR
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    torch.set_num_threads(threads)
    o = OracleHmr(synth.make_hmr_state_dict(TOKENHMR), TOKENHMR, bf16=False)
    p = OracleRtmpose(synth.make_rtmpose_state_dict(RTMPOSE_L), RTMPOSE_L, bf16=False)
    y = OracleYolox(synth.make_yolox_state_dict(YOLOX_L), YOLOX_L, bf16=False) if detector else None
    frames = synth.make_frames(99, 4)
    full = [[0.0, 0.0, 256.0, 256.0]] * frames.shape[0]
    n, used_h, used_p = 0, 0.0, 0.0
    while used_h + used_p < seconds or n == 0:
        t0 = time.perf_counter()
        o.forward(frames)
        t1 = time.perf_counter()
        if y is not None:
            y.forward(frames)
        p.simcc(frames, list(range(frames.shape[0])), full)
        used_p += time.perf_counter() - t1
        used_h += t1 - t0
        n += frames.shape[0]
    fps = n / (used_h + used_p)
    return {"value": fps / 32.0, "unit": "videos/s", "cores": threads, "kind": "port",
            "sample": f"{n} frames through oracle/hmr.py (fp32 torch ViT-H/16 + decoder head) and oracle/dwpose.py "
                      f"({'fp32 torch YOLOX-L + ' if y is not None else ''}RTMPose-l whole-body), {threads} threads, "
                      f"{used_h:.1f} + {used_p:.1f} s = "
                      f"{fps:.3f} frames/s, / 32 frames per clip (the scoring stages, ~450 clips/s on the same host in "
                      f"the config-2 baseline, are <0.1% of this and not added)"}


def run(args, world, rank, dev, metric, allreduce_sum, make_clips):
    from vge import eval as VE
    from vge import ops, synth
    from vge.data import ACTION_CLASSES, pack_frame_store
    from vge.dist import shard
    from vge.dwpose import RTMPOSE_L, YOLOX_L, DwposeExtractor, YoloxDetector
    from vge.extract import single_person_mask
    from vge.hmr import TOKENHMR, HmrExtractor, crop_persons

    C, T = args.clips, 32
    F = C * T
    FC = min(F, max(1, getattr(args, "chunk_clips", 32)) * T)   # frames per extraction pass
    t_setup = time.perf_counter()
    # scoring model, stats and centroids from the (sharded) pre-extracted real set, as in config 2
    n_real_per_class, T_real = 8, 64
    real_idx = shard(list(range(10 * n_real_per_class)), rank, world)
    real_clips = [make_clips(synth.SEED_REAL, i, 1, T_real)[0] for i in real_idx]
    real_cls = [ACTION_CLASSES[i // n_real_per_class] for i in real_idx]
    real_store = ops.DeviceFrameStore.from_host(pack_frame_store(real_clips, [f"r{i}" for i in real_idx], real_cls), dev)
    sums = torch.zeros((2, ops.FEAT_DIM), device=dev, dtype=torch.float64)
    counts = np.zeros(2, np.int64)
    ops.stats_accumulate(real_store, range(real_store.n_videos), sums, counts)
    sums = allreduce_sum(sums, world)
    counts = allreduce_sum(torch.tensor(counts, device=dev), world).cpu().numpy()
    mean, std = ops.stats_finalize(sums, counts)
    enc = ops.Encoder(synth.make_state_dict(synth.DIMS_RAW, synth.DIMS_DIFF), device=dev, compute="f32x3")
    enc.reserve(max(C, 64))
    real_win = torch.tensor([[v, s] for v in range(real_store.n_videos) for s in range(0, T_real - T + 1, 8)],
                            dtype=torch.int32, device=dev)
    stats = VE.ModalityStatsGPU(mean, std, sums, counts)
    rseq, _, _ = VE.encode_windows(enc, real_store, real_win, stats, batch=256)
    label = {c: i for i, c in enumerate(ACTION_CLASSES)}
    y = torch.tensor([label[real_cls[v]] for v in range(real_store.n_videos) for _ in range(0, T_real - T + 1, 8)],
                     dtype=torch.int32, device=dev)
    csum, ccnt = torch.zeros((10, 256), device=dev), torch.zeros((10,), device=dev)
    ops.centroid_accumulate(rseq, y, csum, ccnt)
    centroids = ops.centroid_finalize(allreduce_sum(csum, world), allreduce_sum(ccnt, world))

    # extractors + generated clips: frames resident in HBM; the frame store's SMPL / token arrays (TokenHMR) and
    # keypoint rows (DWPose, whole-frame boxes) are written by the extractors every step
    hsd = synth.make_hmr_state_dict(TOKENHMR)
    ex = HmrExtractor(hsd, TOKENHMR, device=dev, max_frames=FC)
    del hsd
    dw = DwposeExtractor(synth.make_rtmpose_state_dict(RTMPOSE_L), RTMPOSE_L, device=dev, max_instances=2 * FC)
    det = None if args.no_detector else YoloxDetector(synth.make_yolox_state_dict(YOLOX_L), YOLOX_L, device=dev,
                                                      chunk=min(FC, 64))
    no_box = np.zeros(FC, np.int32)
    base = torch.from_numpy(synth.make_frames(1000 + rank, FC)).to(dev)
    if F == FC:
        frames = base
    else:  # distinct frames for every pass, derived on the device from one pass's worth of generated frames
        frames = torch.empty((F,) + tuple(base.shape[1:]), dtype=torch.uint8, device=dev)
        for f0 in range(0, F, FC):
            n = min(FC, F - f0)
            frames[f0:f0 + n] = ((base[:n].to(torch.int16) + (f0 // FC) * 37) % 256).to(torch.uint8)
        del base
    gen_clips = make_clips(synth.SEED_GEN, rank * C, C, T)
    names = [synth.generated_name(rank * C + i) for i in range(C)]
    gstore = ops.DeviceFrameStore.from_host(pack_frame_store(gen_clips, names, ["X"] * C), dev)
    outs = {"pose": gstore.pose, "global_orient": gstore.gori, "betas": gstore.betas, "vit": gstore.vit}
    windows = torch.tensor([[v, 0] for v in range(C)], dtype=torch.int32, device=dev)
    first = torch.arange(C + 1, dtype=torch.int32, device=dev)
    vcls = torch.tensor([label[ACTION_CLASSES[((rank * C + i) // 5) % 10]] for i in range(C)], dtype=torch.int32,
                        device=dev)
    feats = torch.empty((C, T, ops.FEAT_DIM), device=dev)
    host_ac = torch.empty((C,), dtype=torch.float32, pin_memory=True)
    host_tc = torch.empty((C,), dtype=torch.float64, pin_memory=True)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t_setup

    assert tuple(gstore.kp.shape) == (F, 120)
    # the two extractors are independent until the frame store is complete: TokenHMR on one HIP stream, DWPose on
    # another (the detector's host round trip waits on its own stream only), so each fills the other's tails
    s_hmr, s_pose = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    concurrent = not getattr(args, "serial_extract", False)

    Hf, Wf = int(frames.shape[1]), int(frames.shape[2])
    whole = np.tile(np.array([0, 0, Wf, Hf], np.float32), (FC, 1))
    pin_b = torch.empty((FC, 2, 4), dtype=torch.float32, pin_memory=True)
    pin_n = torch.empty((FC,), dtype=torch.int32, pin_memory=True)
    pin_s = torch.empty((FC, 2), dtype=torch.float32, pin_memory=True)
    gate = {"frames": 0, "single_person": 0}

    def detect(fr):
        """the shared person detection -> host (the pose model's instance table and the TokenHMR gate / crop boxes
        are built on the host, as the reference's numpy NMS output is)"""
        n = int(fr.shape[0])
        if det is None:
            return None, no_box[:n], whole[:n]
        boxes, npers, scores = det.detect(fr, with_scores=True)
        pin_b[:n].copy_(boxes, non_blocking=True)
        pin_n[:n].copy_(npers, non_blocking=True)
        pin_s[:n].copy_(scores, non_blocking=True)
        torch.cuda.current_stream(dev).synchronize()
        hb, hn = pin_b[:n].numpy(), pin_n[:n].numpy()
        keep = single_person_mask(pin_s[:n].numpy())
        gate["frames"] += n
        gate["single_person"] += int(keep.sum())
        return hb, hn, np.where(keep[:, None], hb[:, 0], whole[:n])

    def hmr(fr, hbox, f0):
        crops = crop_persons(fr, hbox)
        ex.extract(crops, out={k: v[f0:f0 + int(fr.shape[0])] for k, v in outs.items()})

    def keypoints(fr, hb, hn, f0):
        dw.keypoints(fr, hb, hn, out=gstore.kp[f0:f0 + int(fr.shape[0])])

    def step():
        for f0 in range(0, F, FC):
            fr = frames[f0:f0 + FC]
            hb, hn, hbox = detect(fr)
            if concurrent:
                cur = torch.cuda.current_stream(dev)
                s_hmr.wait_stream(cur)
                s_pose.wait_stream(cur)
                with torch.cuda.stream(s_hmr):
                    hmr(fr, hbox, f0)
                with torch.cuda.stream(s_pose):
                    keypoints(fr, hb, hn, f0)
                cur.wait_stream(s_hmr)
                cur.wait_stream(s_pose)
            else:
                hmr(fr, hbox, f0)
                keypoints(fr, hb, hn, f0)
        ops.featurize(gstore, windows, stats.mean, stats.std, out=feats)
        seq, _, tcw = enc.encode(feats, frame_embed=False, tc=True)
        ac, tc = ops.score_videos(seq, tcw, first, vcls, centroids)
        host_ac.copy_(ac, non_blocking=True)
        host_tc.copy_(tc, non_blocking=True)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # per-kernel hipEvents inside concurrent streams would time shared GPU wall time, so with concurrent extractors
    # the stage / roofline events are recorded on serial steps right after the timed region instead
    n_chunks = -(-F // FC)
    prof_steps = args.steps if n_chunks == 1 else 1   # large runs: one serial profiled step
    if not concurrent:
        ex.profile_begin(prof_steps * n_chunks)
        dw.profile_begin(prof_steps * n_chunks)
        if det is not None:
            det.profile_begin(prof_steps * n_chunks)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    dt_t = torch.tensor([dt], dtype=torch.float64, device=dev if dist.is_initialized() and
                        dist.get_backend() == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
    dt = float(dt_t.item())
    if concurrent:
        ex.profile_begin(prof_steps * n_chunks)
        dw.profile_begin(prof_steps * n_chunks)
        if det is not None:
            det.profile_begin(prof_steps * n_chunks)
        concurrent = False
        for _ in range(prof_steps):
            step()
        torch.cuda.synchronize()
        concurrent = True
    st, ncalls, gemm_flops_per_frame = ex.profile_read()
    dst, dcalls, dw_flops = dw.profile_read()
    yst, ycalls, y_flops = det.profile_read() if det is not None else ({}, 0, 0.0)
    assert np.isfinite(host_ac.numpy()).all() and np.isfinite(host_tc.numpy()).all()
    if rank != 0:
        return None
    n = max(ncalls, 1)
    gemm_ms = st["gemm"] / n
    achieved = gemm_flops_per_frame * FC / (gemm_ms * 1e-3) / 1e12
    out = {
        "metric": metric,
        "value": world * C * args.steps / dt,
        "unit": "videos/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16 (extractor: bf16 operands, f32 accumulate / residual stream) + f32x3 (scorer)",
        "data": "synthetic 256x256 RGB frames (vge.synth.make_frames); random-init weights of the TokenHMR "
                "(ViT-H/16 + decoder), YOLOX-L, RTMPose-l whole-body and scorer architectures",
        "config": {"workload": "BASELINE config 3: TokenHMR + DWPose (YOLOX-L + RTMPose-l) extract -> featurise -> "
                               "encoder -> AC/TC, 32-frame 256x256 clips, full frames resident in HBM (one YOLOX-L "
                               "detection per frame for DWPose and TokenHMR's single-person gate; ViTDetDataset crops)"
                               + (" [--no-detector: whole-frame boxes]" if det is None else ""),
                   "clips_per_gpu": C, "frames_per_step_per_gpu": F, "frames_per_extraction_pass": FC,
                   "parallelism": f"video-sharded x{world}"},
        "roofline": {"bound": "mfma", "kernel": "gemm_bf16_kernel (ViT-H/16 backbone: patch-embed, qkv, proj, fc1, "
                                                "fc2; dense bf16 MFMA peak)",
                     "achieved": achieved, "peak": BF16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / BF16_MFMA_PEAK_TFLOPS, "traffic": None,
                     "flop_per_call": gemm_flops_per_frame * FC, "gemm_ms_per_call": gemm_ms},
        "stage_ms": {**{f"hmr_{k}": v / n for k, v in st.items()},
                     **{f"dwpose_{k}": v / max(dcalls, 1) for k, v in dst.items()},
                     **{f"yolox_{k}": v / max(ycalls, 1) for k, v in yst.items()}},
        "yolox_gemm_tflops": (y_flops / (yst["gemm"] / ycalls * 1e-3) / 1e12) if ycalls else None,
        "dwpose_gemm_tflops": dw_flops / (dst["gemm"] / max(dcalls, 1) * 1e-3) / 1e12,
        "frames_per_s": world * F * args.steps / dt,
        "front_end": {"detector": "YOLOX-L (stand-in for detectron2 Faster R-CNN X101-FPN)" if det is not None else None,
                      "gate": "exactly one person box with score > 0.5 (mesh_generator.py:103-111)",
                      "single_person_fraction": (gate["single_person"] / gate["frames"]) if gate["frames"] else None,
                      "crop": "ViTDetDataset warp to 256x256 (vge_hmr_crop); gate-rejected frames take the whole "
                              "frame, so every frame is extracted"},
        "extractors": ("concurrent (TokenHMR and DWPose on two HIP streams; stage_ms / roofline from hipEvents on "
                       "serial steps after the timed region)") if concurrent else "serial",
        "setup_s": setup_s,
    }
    out["cpu_baseline"] = None if (world > 1 or args.no_cpu_baseline) else cpu_baseline_e2e(args.cpu_seconds, det is not None)
    return out
