"""BASELINE config 4 end to end as ONE sharded job: variable-length videos' frames -> the extraction chain on each
rank's shard (detectron2 Faster R-CNN gate + TokenHMR, YOLOX-L + DWPose; vge.extract.extract_videos, passes of up to
32 frames packing several videos) -> npz / keypoints.npy in the reference's generated-set layout -> the video-sharded
eval flow (vge.dist.run_eval_distributed: stats / centroid sufficient statistics exchanged, scores gathered to rank 0).
Two ranks (gloo collectives, both on the box's one GPU).  Rank 0's merged scores must equal, within the north star's
1e-4, oracle/evalflow.py's eval.py restatement over the files the ranks wrote; the rejected video (fewer than 80 %
single-person frames, mesh_generator.py:113-117) gets keypoints but no npz and no score.  TokenHMR runs 2 of ViT-H's 32
blocks (full width); parity of the networks vs the upstream weights is unpinned."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

LENS = (10, 14, 12, 16, 10, 12, 14, 18)      # frames per video; the last one is rejected (5 of 18 frames bad)
BAD = (1, 2, 1, 2, 1, 2, 1, 5)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _plan():
    from vge.data import ACTION_CLASSES
    return [f"vgen_{ACTION_CLASSES[k % 6]}_{k:02d}" for k in range(len(LENS))]


def _rank_main(rank, ws, port, paths, ckpt, root, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from vge import dist as VD
    from vge import synth
    from vge.dwpose import RTMPOSE_L, YOLOX_L, DwposeExtractor, Wholebody, YoloxDetector
    from vge.extract import extract_videos, gate_mask
    from vge.frcnn import FRCNN_X101, FrcnnDetector
    from vge.hmr import HmrConfig, HmrExtractor
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        dev = torch.device("cuda:0")
        hcfg = HmrConfig(depth=2)
        hmr = HmrExtractor(synth.make_hmr_state_dict(hcfg), hcfg, device=dev, max_frames=32)
        gdet = FrcnnDetector(synth.make_gate_frcnn_state_dict(FRCNN_X101), FRCNN_X101, device=dev, chunk=32)
        wb = Wholebody(YoloxDetector(synth.make_gate_detector_state_dict(YOLOX_L), YOLOX_L, device=dev, chunk=32),
                       DwposeExtractor(synth.make_rtmpose_state_dict(RTMPOSE_L), RTMPOSE_L, device=dev,
                                       max_instances=64))
        pool = torch.from_numpy(synth.make_frame_pool(4242, 512)).to(dev)
        one = gate_mask(gdet.detect(pool)["n_person"].cpu().numpy())
        good, bad = np.flatnonzero(one), np.flatnonzero(~one)
        rs = np.random.default_rng(17)
        stems = _plan()
        videos = []
        for k, (T, nb) in enumerate(zip(LENS, BAD)):   # every rank draws the same plan; each keeps its shard
            sel = rs.permutation(np.concatenate([rs.choice(bad, nb, replace=False), rs.choice(good, T - nb, replace=False)]))
            videos.append((stems[k], sel))
        mine = VD.shard(videos, rank, ws)
        wrote = extract_videos(hmr, wb, gdet, [(s, pool[torch.from_numpy(i).to(dev)].contiguous()) for s, i in mine],
                               root + "/generated_meshes", root + "/generated_kps", max_frames=32)
        dist.barrier()   # every rank's files are on disk before any rank scans the generated set
        res = VD.run_eval_distributed(root + "/generated_meshes", paths["real"], ckpt, root + "/generated_kps",
                                      paths["real_kp"], out_json=None, device=dev)
        q.put((rank, res, wrote))
    finally:
        dist.destroy_process_group()


def test_sharded_extraction_and_scoring_match_the_oracle_flow(golden_dataset, tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import evalflow
    from vge import synth
    paths, ckpt = golden_dataset
    root = str(tmp_path)
    ws = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, ws, port, paths, ckpt, root, q)) for r in range(ws)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=420)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = dict((r, (res, wrote)) for r, res, wrote in (q.get() for _ in range(ws)))
    merged = got[0][0]
    assert got[1][0] is None
    wrote = {**got[0][1], **got[1][1]}
    stems = _plan()
    assert sorted(wrote) == sorted(stems)
    assert wrote[stems[-1]] is None and all(wrote[s] for s in stems[:-1])   # the 80 % rule
    assert all(os.path.exists(os.path.join(root, "generated_kps", s, "keypoints.npy")) for s in stems)
    ref, _ = evalflow.run_eval(paths["real"], paths["real_kp"], root + "/generated_meshes", root + "/generated_kps",
                               synth.make_state_dict(synth.DIMS_RAW, synth.DIMS_DIFF), synth.DIMS_RAW, synth.DIMS_DIFF)
    assert sorted(merged) == sorted(ref) == sorted(stems[:-1])
    worst = max(abs(merged[v][k] - ref[v][k]) for v in ref for k in ref[v])
    for v in ref:
        assert sorted(merged[v]) == sorted(ref[v])
    print(f"config-4 chain (2 ranks): {len(ref)} videos scored, max|gpu - oracle| {worst:.2e}")
    assert worst < 1e-4, worst
