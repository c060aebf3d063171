"""End-to-end workload of bench.py (`--workload e2e`, BASELINE.json configs[2]): 256x256 RGB frames resident in HBM
-> TokenHMR extractor (ViT-H/16 backbone + SMPL token-decoder head, bf16 MFMA; vge_hmr.h) and DWPose keypoints
(RTMPose-l whole-body, bf16 MFMA implicit-GEMM convs; vge_dwpose.h) writing the frame store -> featurise ->
fusion encoder (f32x3) -> AC/TC, per step `--clips` 32-frame clips per GPU.

The reference pipeline is extract_mesh.py (TokenHMR per frame, modifications/mesh_generator.py:119-171) + DWPose
(modifications/process_video.py) -> npz / keypoints.npy on disk -> eval.py.  Here the frames-to-scores path stays
in HBM and both extractors start from the full frames, each with the reference's own person detector on every frame:
TokenHMR's front end (mesh_generator.py:101-145) runs detectron2's Faster R-CNN X101-32x8d-FPN at 800 px (vge.frcnn),
applies the single-person gate (exactly one person instance > 0.5 per frame, >= 80 % of a video's frames) and crops
the kept frames with ViTDetDataset's warp (vge_hmr_crop); DWPose runs as the reference's Wholebody does (YOLOX-L
persons, RTMPose-l on persons 0 / 1, the whole frame when nobody is found -> keypoints.npy rows).  The Faster R-CNN +
TokenHMR chain runs on one HIP stream, YOLOX + DWPose on another.  `--no-detector`: neither detector (whole-frame
boxes, every frame kept).  Parity for the upstream models is unpinned.

Roofline: the backbone GEMMs (MFMA bound: hipBLASLt for the bias / f32-residual linears, gemm_bf16_kernel for the GELU
and position-embedding ones; vge_blaslt.cpp): achieved = algorithmic FLOPs of every backbone GEMM launch / their
summed durations (hipEvents recorded around each launch on the extract stream inside the timed
steps); peak = dense bf16 MFMA 2516.6 TFLOP/s.  cpu_baseline = oracle/hmr.py (the fp32 torch restatement of the
same ViT-H + head) + the scoring restatement on this host, bounded sample.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

BF16_MFMA_PEAK_TFLOPS = 2516.6
# kernel sources whose PMC pass (tools/profile_e2e.sh -> tools/pmc_e2e.py -> profiles/pmc_e2e.json) gives `traffic`
E2E_KERNEL_SOURCES = {"gemm_bf16_kernel": ["vge_vit.hip", "vge_blaslt.cpp", "vge_hmr.cpp"],
                      "yolox_conv": ["vge_cnn.hip", "vge_cnn_host.h", "vge_yolox.cpp", "vge_vit.hip", "vge_blaslt.cpp"],
                      "frcnn_conv": ["vge_cnn.hip", "vge_cnn_host.h", "vge_frcnn.cpp", "vge_vit.hip", "vge_gconv.hip",
                                     "vge_blaslt.cpp", "vge_frcnn_kernels.hip"]}  # (the fused stem + pool)
YOLOX_CHUNK = 1024  # frames per detector pass: the whole extraction pass (tools/yolox_prof.py --chunk: 246.4 / 238.7 / 234.5 ms per 1,024 frames at 256 / 512 / 1,024, profiles/ab_r06ax_chunks.json)
# frames per Faster R-CNN workspace chunk (~0.3 GB per 800 x 800 frame): 64 was -6 % vs 32 (profiles/ab_r05m_*); 128,
# possible since the 1x1 convs' GEMM epilogue addresses through 64-bit offsets, -1.2 % vs 64 (profiles/ab_r06b_frcnn_chunk.json)
FRCNN_CHUNK = 256  # 197.2 -> 193.6 ms per 256 frames vs 128 (profiles/ab_r06ax_chunks.json)


def e2e_traffic(kernel: str, frames: float):
    """HBM bytes (FETCH_SIZE x 2 + WRITE_SIZE) of `frames` frames through `kernel` from the committed PMC pass, only
    while the kernel's sources hash to the pass's `source_sha`; else None."""
    from pathlib import Path
    from bench import sources_sha
    try:
        e = json.loads((Path(__file__).resolve().parent / "profiles" / "pmc_e2e.json").read_text())[kernel]
        if e.get("source_sha") != sources_sha(E2E_KERNEL_SOURCES[kernel]):
            return None
        return e["hbm_bytes_per_frame"] * frames
    except (OSError, KeyError, ValueError):
        return None


def cpu_baseline_e2e(seconds: float, detector: bool = True):
    from oracle.dwpose import OracleRtmpose
    from oracle.frcnn import OracleFrcnn
    from oracle.hmr import OracleHmr
    from oracle.yolox import OracleYolox
    from vge import synth
    from vge.dwpose import RTMPOSE_L, YOLOX_L
    from vge.frcnn import FRCNN_X101
    from vge.hmr import TOKENHMR
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    torch.set_num_threads(threads)
    o = OracleHmr(synth.make_hmr_state_dict(TOKENHMR), TOKENHMR, bf16=False)
    p = OracleRtmpose(synth.make_rtmpose_state_dict(RTMPOSE_L), RTMPOSE_L, bf16=False)
    y = OracleYolox(synth.make_yolox_state_dict(YOLOX_L), YOLOX_L, bf16=False) if detector else None
    g = OracleFrcnn(synth.make_gate_frcnn_state_dict(FRCNN_X101), FRCNN_X101, bf16=False) if detector else None
    frames = synth.make_frames(99, 4)
    full = [[0.0, 0.0, 256.0, 256.0]] * frames.shape[0]
    n, used_h, used_p, used_g, ng = 0, 0.0, 0.0, 0.0, 0
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
    if g is not None:   # the gate detector: one frame (several seconds of CPU work at 800 px), rate per frame
        t0 = time.perf_counter()
        g.detect(frames[:1])
        used_g, ng = time.perf_counter() - t0, 1
    spf = (used_h + used_p) / n + (used_g / ng if ng else 0.0)
    fps = 1.0 / spf
    return {"value": fps / 32.0, "unit": "videos/s", "cores": threads, "kind": "port",
            "sample": f"{n} frames through oracle/hmr.py (fp32 torch ViT-H/16 + decoder head) and oracle/dwpose.py "
                      f"({'fp32 torch YOLOX-L + ' if y is not None else ''}RTMPose-l whole-body) in "
                      f"{used_h:.1f} + {used_p:.1f} s"
                      + (f", {ng} frame through oracle/frcnn.py (fp32 torch Faster R-CNN X101-32x8d-FPN at 800 px) in "
                         f"{used_g:.1f} s" if ng else "")
                      + f", {threads} threads: {fps:.3f} frames/s, / 32 frames per clip (the scoring stages, ~450 "
                        f"clips/s on the same host in the config-2 baseline, are <0.1% of this and not added)"}


def run(args, world, rank, dev, metric, allreduce_sum, make_clips):
    from vge import eval as VE
    from vge import ops, synth
    from vge.data import ACTION_CLASSES, pack_frame_store
    from vge.dist import shard
    from vge.dwpose import RTMPOSE_L, YOLOX_L, DwposeExtractor, YoloxDetector
    from vge.extract import gate_mask, gate_videos
    from vge.frcnn import FRCNN_X101, FrcnnDetector
    from vge.hmr import TOKENHMR, HmrExtractor, crop_persons

    C, T = args.clips, 32
    F = C * T
    FC = min(F, max(1, getattr(args, "chunk_clips", 32)) * T)   # frames per extraction pass
    t_setup = time.perf_counter()
    if rank == 0:  # a progress line every 30 s for the whole run (setup and warm-up print nothing else for minutes)
        import threading

        def _alive():
            while True:
                time.sleep(30.0)
                print(f"[e2e] running, {time.perf_counter() - t_setup:.0f} s", file=sys.stderr, flush=True)
        threading.Thread(target=_alive, daemon=True).start()
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
    det = None if args.no_detector else YoloxDetector(synth.make_gate_detector_state_dict(YOLOX_L), YOLOX_L,
                                                      device=dev, chunk=min(FC, YOLOX_CHUNK))
    gdet = None if args.no_detector else FrcnnDetector(synth.make_gate_frcnn_state_dict(FRCNN_X101), FRCNN_X101,
                                                       device=dev, chunk=min(FC, FRCNN_CHUNK))
    no_box = np.zeros(FC, np.int32)
    Hf = Wf = 256
    whole = np.tile(np.array([0, 0, Wf, Hf], np.float32), (FC, 1))
    # the generated clips' frames: drawn from a pool of synthetic scenes by what the gate detector finds in each pool
    # frame (setup, untimed), so that 9 clips in 10 pass the single-person gate (2-3 of their 32 frames with no or two
    # persons) and 1 in 10 is rejected (12 such frames: 20 / 32 < 80 %).  The timed steps run the detectors on every
    # frame again and take every decision from their output.
    gate_plan = {"accept_every": 10, "bad_frames_accepted": (2, 3), "bad_frames_rejected": 12}
    if det is None:
        frames = torch.from_numpy(synth.make_frame_pool(5000 + 997 * rank, min(F, 4096))).to(dev)
        frames = frames[torch.arange(F, device=dev) % frames.shape[0]] if F > frames.shape[0] else frames
    else:
        P = 2048
        pool = torch.from_numpy(synth.make_frame_pool(5000 + 997 * rank, P)).to(dev)
        good = np.flatnonzero(gate_mask(gdet.detect(pool)["n_person"].cpu().numpy()))
        bad = np.setdiff1d(np.arange(P), good)
        if good.size < 64 or bad.size < 64:
            raise RuntimeError(f"e2e: the gate detector finds exactly one person in {good.size} of {P} pool frames; "
                               "recalibrate vge.synth.GATE_FRCNN_BG (tools/frcnn_gate_calib.py)")
        rs = np.random.default_rng(11 + rank)
        idx = np.empty(F, np.int64)
        for c in range(C):
            nb = (gate_plan["bad_frames_rejected"] if c % gate_plan["accept_every"] == gate_plan["accept_every"] - 1
                  else gate_plan["bad_frames_accepted"][c % 2])
            sel = np.concatenate([rs.choice(bad, nb), rs.choice(good, T - nb)])
            idx[c * T:(c + 1) * T] = rs.permutation(sel)
        frames = pool[torch.from_numpy(idx).to(dev)]
        del pool
    gen_clips = make_clips(synth.SEED_GEN, rank * C, C, T)
    names = [synth.generated_name(rank * C + i) for i in range(C)]
    gstore = ops.DeviceFrameStore.from_host(pack_frame_store(gen_clips, names, ["X"] * C), dev)
    outs = {"pose": gstore.pose, "global_orient": gstore.gori, "betas": gstore.betas, "vit": gstore.vit}
    vcls_all = np.array([label[ACTION_CLASSES[((rank * C + i) // 5) % 10]] for i in range(C)], np.int32)
    feats = torch.empty((C, T, ops.FEAT_DIM), device=dev)
    host_ac = torch.empty((C,), dtype=torch.float32, pin_memory=True)
    host_tc = torch.empty((C,), dtype=torch.float64, pin_memory=True)
    # per step: the accepted videos' frame-store descriptors {frame_off, n_frames, kp_off, kp_frames} (the npz holds
    # the kept frames only, keypoints.npy every frame: extract_mesh.py:35-43, process_video.py:71-84), windows, the
    # per-video window ranges and classes -> one pinned host table, one copy
    pin_tab = torch.empty((C * 4 + C * 2 + (C + 1) + C,), dtype=torch.int32, pin_memory=True)
    dev_tab = torch.empty_like(pin_tab, device=dev)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t_setup

    assert tuple(gstore.kp.shape) == (F, 120) and tuple(frames.shape) == (F, Hf, Wf, 3)
    # the two extractors are independent until the frame store is complete: TokenHMR on one HIP stream, DWPose on
    # another (the detector's host round trip waits on its own stream only), so each fills the other's tails
    s_hmr, s_pose = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    concurrent = not getattr(args, "serial_extract", False)

    pin_b = torch.empty((FC, 2, 4), dtype=torch.float32, pin_memory=True)
    pin_n = torch.empty((FC,), dtype=torch.int32, pin_memory=True)
    pin_gb = torch.empty((FC, 2, 5), dtype=torch.float32, pin_memory=True)
    pin_gn = torch.empty((FC,), dtype=torch.int32, pin_memory=True)
    gate_ready = torch.cuda.Event()
    gate = {"frames": 0, "single_person": 0, "videos": 0, "accepted": 0, "hmr_frames": 0}

    def detect_gate(fr):
        """the Faster R-CNN on every frame, its person outputs to pinned host memory (the gate and the crop boxes are
        decided on the host, as mesh_generator.py does with the predictor's instances)"""
        n = int(fr.shape[0])
        if gdet is None:
            return
        g = gdet.detect(fr)
        pin_gb[:n].copy_(g["person"], non_blocking=True)
        pin_gn[:n].copy_(g["n_person"], non_blocking=True)
        gate_ready.record()

    def gate_result(n):
        """-> (person boxes [n, 4] of the first class-0 instance, single-person mask) once the gate's copies landed"""
        if gdet is None:
            return None, np.ones(n, bool)
        gate_ready.synchronize()
        keep = gate_mask(pin_gn[:n].numpy())
        gate["frames"] += n
        gate["single_person"] += int(keep.sum())
        return pin_gb[:n, 0, :4].numpy(), keep

    def detect_pose(fr):
        """DWPose's YOLOX persons -> host (the pose model's instance table, as the reference's numpy NMS output)"""
        n = int(fr.shape[0])
        if det is None:
            return None, no_box[:n]
        boxes, npers = det.detect(fr)
        pin_b[:n].copy_(boxes, non_blocking=True)
        pin_n[:n].copy_(npers, non_blocking=True)
        torch.cuda.current_stream(dev).synchronize()
        return pin_b[:n].numpy(), pin_n[:n].numpy()

    def hmr(fr, gb, kept, off):
        """TokenHMR on the kept frames of the pass's accepted videos, into rows off.. of the frame store"""
        nk = int(kept.size)
        if nk:
            box = whole[:nk] if gb is None else gb[kept]
            crops = crop_persons(fr, box, kept)
            ex.extract(crops, out={k: v[off:off + nk] for k, v in outs.items()})
            gate["hmr_frames"] += nk

    def keypoints(fr, hb, hn, f0):
        dw.keypoints(fr, hb, hn, out=gstore.kp[f0:f0 + int(fr.shape[0])])

    beat = [time.perf_counter()]

    def heartbeat(msg):
        """a progress line every ~20 s on stderr (a 1k-clip step runs for about a minute without other output)"""
        now = time.perf_counter()
        if now - beat[0] > 20.0:
            beat[0] = now
            print(f"[e2e] {msg}", file=sys.stderr, flush=True)

    def step():
        tab = pin_tab.numpy()
        vids = tab[:4 * C].reshape(C, 4)
        acc = []
        off = 0
        cur = torch.cuda.current_stream(dev)
        if concurrent:
            s_hmr.wait_stream(cur)
            s_pose.wait_stream(cur)
        for f0 in range(0, F, FC):
            fr = frames[f0:f0 + FC]
            n = int(fr.shape[0])
            # Faster R-CNN on the TokenHMR stream while YOLOX + DWPose run on the other; the host waits for the gate
            # only after DWPose is queued, so chunk i's TokenHMR overlaps chunk i + 1's YOLOX + DWPose
            with torch.cuda.stream(s_hmr if concurrent else cur):
                detect_gate(fr)
            with torch.cuda.stream(s_pose if concurrent else cur):
                hb, hn = detect_pose(fr)
                keypoints(fr, hb, hn, f0)
            gb, keep = gate_result(n)
            # mesh_generator.py:101-117 per video: the frames with exactly one person; the video is rejected
            # (process_video returns False, no npz) when they are fewer than 80 % of its frames
            c0 = f0 // T
            va, kept, desc = gate_videos(keep, T, off)
            gate["videos"] += n // T
            if va.size:
                desc[:, 2] += f0   # keypoint rows of the batch's videos sit at their frame offsets
                vids[len(acc):len(acc) + va.size] = desc
                acc.extend((va + c0).tolist())
            with torch.cuda.stream(s_hmr if concurrent else cur):
                hmr(fr, gb, kept, off)
            off += int(kept.size)
            heartbeat(f"extraction pass {f0 // FC + 1} / {-(-F // FC)}")
        if concurrent:
            cur.wait_stream(s_hmr)
            cur.wait_stream(s_pose)
        nA = len(acc)
        gate["accepted"] += nA
        if nA == 0:
            return
        # eval.py:360-400 on the accepted videos (window start 0: T' <= 32 frames, _slice_or_pad pads)
        win = tab[4 * C:4 * C + 2 * nA].reshape(nA, 2)
        win[:, 0], win[:, 1] = np.arange(nA), 0
        first = tab[6 * C:6 * C + nA + 1]
        first[:] = np.arange(nA + 1)
        vc = tab[7 * C + 1:7 * C + 1 + nA]
        vc[:] = vcls_all[acc]
        dev_tab.copy_(pin_tab, non_blocking=True)
        gstore.videos[:nA].copy_(dev_tab[:4 * nA].view(nA, 4))
        windows = dev_tab[4 * C:4 * C + 2 * nA].view(nA, 2)
        ops.featurize(gstore, windows, stats.mean, stats.std, out=feats[:nA])
        seq, _, tcw = enc.encode(feats[:nA], frame_embed=False, tc=True)
        ac, tc = ops.score_videos(seq, tcw, dev_tab[6 * C:6 * C + nA + 1], dev_tab[7 * C + 1:7 * C + 1 + nA],
                                  centroids)
        host_ac[:nA].copy_(ac, non_blocking=True)
        host_tc[:nA].copy_(tc, non_blocking=True)
        if gdet is None:  # else the next step's first gate result syncs behind this step before the table is rewritten
            torch.cuda.current_stream(dev).synchronize()

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
            gdet.profile_begin(prof_steps * n_chunks)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    hmr_frames0 = gate["hmr_frames"]
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
    gate_timed = dict(gate)
    # every extract / keypoints / detect call of the profiled steps is recorded (at most one per pass each)
    if concurrent:
        ex.profile_begin(prof_steps * n_chunks)
        dw.profile_begin(prof_steps * n_chunks)
        if det is not None:
            det.profile_begin(prof_steps * n_chunks)
            gdet.profile_begin(prof_steps * n_chunks)
    # TokenHMR frames of one step (the same every step: the clips and the detector are deterministic)
    hmr_frames_step = (gate["hmr_frames"] - hmr_frames0) / args.steps
    if concurrent:
        concurrent = False
        for _ in range(prof_steps):
            step()
        torch.cuda.synchronize()
        concurrent = True
    prof_hmr_frames = hmr_frames_step * prof_steps
    st, ncalls, gemm_flops_per_frame = ex.profile_read()
    dst, dcalls, dw_flops = dw.profile_read()
    yst, ycalls, y_flops = det.profile_read() if det is not None else ({}, 0, 0.0)
    gst, gcalls, g_flops = gdet.profile_read() if gdet is not None else ({}, 0, (0.0, 0.0))
    assert np.isfinite(host_ac.numpy()).all() and np.isfinite(host_tc.numpy()).all()
    if rank != 0:
        return None
    n = max(ncalls, 1)
    gemm_ms = st["gemm"] / n
    # TokenHMR runs on the kept frames only, so a call's size varies: FLOPs of the recorded calls / their GEMM time
    hmr_frames_per_call = prof_hmr_frames / n
    achieved = gemm_flops_per_frame * prof_hmr_frames / (st["gemm"] * 1e-3) / 1e12 if st["gemm"] else 0.0
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
        "data": "synthetic 256x256 RGB frames (vge.synth.make_frame_pool, drawn by the detector's findings at setup); "
                "random-init weights of the TokenHMR "
                "(ViT-H/16 + decoder), Faster R-CNN X101-32x8d-FPN, YOLOX-L, RTMPose-l whole-body and scorer "
                "architectures",
        "config": {"workload": "BASELINE config 3: TokenHMR (Faster R-CNN X101-FPN gate + ViT-H) + DWPose (YOLOX-L + "
                               "RTMPose-l) extract -> featurise -> encoder -> AC/TC, 32-frame 256x256 clips, full frames "
                               "resident in HBM (every frame through both detectors; ViTDetDataset crops)"
                               + (" [--no-detector: whole-frame boxes]" if det is None else ""),
                   "clips_per_gpu": C, "frames_per_step_per_gpu": F, "frames_per_extraction_pass": FC,
                   "parallelism": f"video-sharded x{world}"},
        "roofline": {"bound": "mfma", "kernel": "ViT-H/16 backbone GEMMs: qkv, proj, fc2 on hipBLASLt, patch-embed and "
                                                "fc1 (GELU) on gemm_bf16_kernel; dense bf16 MFMA peak",
                     "achieved": achieved, "peak": BF16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / BF16_MFMA_PEAK_TFLOPS,
                     "traffic": e2e_traffic("gemm_bf16_kernel", hmr_frames_per_call),
                     "traffic_source": "profiles/pmc_e2e.json (tools/profile_e2e.sh: PMC of the same GEMM dispatches on "
                                       "tools/time_hmr.py, bytes per frame x frames per call)",
                     "flop_per_call": gemm_flops_per_frame * hmr_frames_per_call, "gemm_ms_per_call": gemm_ms,
                     "frames_per_call": hmr_frames_per_call},
        "stage_ms": {**{f"hmr_{k}": v / n for k, v in st.items()},
                     **{f"dwpose_{k}": v / max(dcalls, 1) for k, v in dst.items()},
                     **{f"yolox_{k}": v / max(ycalls, 1) for k, v in yst.items()},
                     **{f"frcnn_{k}": v / max(gcalls, 1) for k, v in gst.items()}},
        "gate_detector": {"model": "detectron2 Faster R-CNN X101-32x8d-FPN (COCO), 800 px, bf16 operands",
                          "gflop_per_frame": (sum(gdet.flops(Hf, Wf)) / 1e9) if gdet is not None else None,
                          "backbone_gemm_tflops": (g_flops[0] / (gst["backbone_gemm"] / gcalls * 1e-3) / 1e12)
                          if gcalls and gst["backbone_gemm"] else None,
                          "head_gemm_tflops": (g_flops[1] / (gst["head_gemm"] / gcalls * 1e-3) / 1e12)
                          if gcalls and gst["head_gemm"] else None,
                          "frac_of_bf16_peak": (g_flops[0] + g_flops[1]) / ((gst["backbone_gemm"] + gst["head_gemm"])
                                                                           / gcalls * 1e-3) / 1e12
                          / BF16_MFMA_PEAK_TFLOPS if gcalls and gst["backbone_gemm"] else None,
                          "traffic_per_call": e2e_traffic("frcnn_conv", FC) if gcalls else None,
                          "chunk_frames": min(FC, FRCNN_CHUNK) if gdet is not None else None},
        "yolox_gemm_tflops": (y_flops / (yst["gemm"] / ycalls * 1e-3) / 1e12) if ycalls else None,
        "yolox_traffic_per_call": e2e_traffic("yolox_conv", FC) if ycalls else None,
        "yolox_chunk_frames": min(FC, YOLOX_CHUNK) if det is not None else None,
        "dwpose_gemm_tflops": dw_flops / (dst["gemm"] / max(dcalls, 1) * 1e-3) / 1e12,
        "frames_per_s": world * F * args.steps / dt,
        "front_end": {"detector": ("detectron2 Faster R-CNN X101-32x8d-FPN (vge.frcnn; "
                                   "vge.synth.make_gate_frcnn_state_dict)") if gdet is not None else None,
                      "dwpose_detector": "YOLOX-L (vge.synth.make_gate_detector_state_dict)" if det is not None else None,
                      "gate": "exactly one person box with score > 0.5 per frame, >= 80 % such frames per video, else "
                              "the video is rejected (mesh_generator.py:101-117)",
                      "single_person_fraction": (gate_timed["single_person"] / gate_timed["frames"])
                      if gate_timed["frames"] else None,
                      "videos_accepted_fraction": (gate_timed["accepted"] / gate_timed["videos"])
                      if gate_timed["videos"] else None,
                      "tokenhmr_frames_per_video": gate_timed["hmr_frames"] / max(gate_timed["videos"], 1),
                      "clip_plan": gate_plan if det is not None else None,
                      "crop": "ViTDetDataset warp to 256x256 (vge_hmr_crop) of the kept frames of accepted videos; "
                              "TokenHMR on those only; DWPose on every frame (process_video.py); rejected videos "
                              "are not scored (no npz)"},
        "extractors": ("concurrent (TokenHMR and DWPose on two HIP streams; stage_ms / roofline from hipEvents on "
                       "serial steps after the timed region)") if concurrent else "serial",
        "setup_s": setup_s,
    }
    out["cpu_baseline"] = None if (world > 1 or args.no_cpu_baseline) else cpu_baseline_e2e(args.cpu_seconds, det is not None)
    return out
