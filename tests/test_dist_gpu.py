"""vge.dist.run_eval_distributed on the GPU: two ranks (gloo collectives, both on cuda:0 of the one-GPU
box) each score their shard through libvge.so; rank 0's merged video_scores.json must match the
single-process reference golden vectors within the north-star tolerance."""
import json
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, ws, port, paths, ckpt, out_json, q, overlap="1"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), VGE_FLOW_OVERLAP=overlap)
    import torch.distributed as dist
    from vge import dist as VD
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        t = {}
        res = VD.run_eval_distributed(paths["generated_meshes"], paths["real"], ckpt, paths["generated_kps"],
                                      paths["real_kp"], out_json=out_json if rank == 0 else None, device="cuda:0",
                                      timings=t)
        q.put((rank, res, t))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ws,overlap", [(2, "1"), (2, "0"), (8, "1")])
def test_two_rank_run_eval_matches_golden(golden_dataset, golden_meta, tmp_path, ws, overlap):
    """Both phase orders: background generated-set decode + checkpoint read (default) and eval.py's serial order; and
    eight ranks (config 4's one rank per GPU of a node, here all on the box's one GPU over gloo)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    paths, ckpt = golden_dataset
    out = str(tmp_path / "video_scores.json")
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, ws, port, paths, ckpt, out, q, overlap)) for r in range(ws)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = dict((r, res) for r, res, _ in (q.get() for _ in range(ws)))
    assert all(got[r] is None for r in range(1, ws))
    merged = got[0]
    ref = golden_meta["video_scores"]
    assert sorted(merged) == sorted(ref)
    worst = max(abs(ref[v][k] - merged[v][k]) for v in ref for k in ref[v])
    assert worst < 1e-4, worst
    assert json.loads(open(out).read()) == merged


@pytest.mark.parametrize("overlap", ["1", "0"])
def test_missing_generated_keypoints_raise_in_either_order(golden_dataset, tmp_path, monkeypatch, overlap):
    """A generated video without keypoints.npy raises FileNotFoundError (utils.py:416-417) from the flow whether its
    decode ran on the background thread or in order."""
    import shutil
    from vge import dist as VD
    paths, ckpt = golden_dataset
    kp = tmp_path / "generated_kps"
    shutil.copytree(paths["generated_kps"], kp)
    victim = sorted(d for d in kp.iterdir() if d.is_dir())[0]
    (victim / "keypoints.npy").unlink()
    monkeypatch.setenv("VGE_FLOW_OVERLAP", overlap)
    with pytest.raises(FileNotFoundError, match="Expected keypoints"):
        VD.run_eval_distributed(paths["generated_meshes"], paths["real"], ckpt, str(kp), paths["real_kp"],
                                out_json=None, device="cuda:0")


def _nccl_main(paths, ckpt, out_json, feats_path, human, q):
    """One rank on an RCCL (nccl) process group: every exchange of the flow runs through RCCL even at world size 1
    (vge.dist.allgather_sum / agree / gather_to_rank0 do not short-circuit inside a group), so host tensors handed
    to a collective would fail here exactly as on 8 GPUs."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    import torch.distributed as dist
    from vge import dist as VD
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        res = VD.run_eval_distributed(paths["generated_meshes"], paths["real"], ckpt, paths["generated_kps"],
                                      paths["real_kp"], out_json=out_json, device="cuda:0", human_scores_path=human,
                                      save_features=feats_path)
        q.put(("ok", res))
    except BaseException as e:  # noqa: BLE001 -- reported to the parent
        q.put(("err", repr(e)))
    finally:
        dist.destroy_process_group()


def test_rccl_flow_matches_golden(golden_dataset, golden_meta, golden_flow, tmp_path):
    """The sharded eval flow on an RCCL group (stats counts are host int64, status flags host int32: both must be
    staged on the GPU), with the distributed CLI's --save-features and --human-scores outputs."""
    import numpy as np
    from pathlib import Path
    paths, ckpt = golden_dataset
    out, feats = str(tmp_path / "video_scores.json"), str(tmp_path / "window_features.pt")
    human = str(Path(__file__).parent / "golden" / "tag_human_scores.json")
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    p = ctx.Process(target=_nccl_main, args=(paths, ckpt, out, feats, human, q))
    p.start()
    p.join(timeout=300)
    assert p.exitcode == 0, p.exitcode
    status, merged = q.get()
    assert status == "ok", merged
    ref = golden_meta["video_scores"]
    assert sorted(merged) == sorted(ref)
    assert max(abs(ref[v][k] - merged[v][k]) for v in ref for k in ref[v]) < 1e-4
    assert json.loads(open(out).read()) == merged
    f = torch.load(feats, weights_only=True)
    assert np.abs(f["seq_embeds"].numpy() - golden_flow["seq_embeds"]).max() < 2e-5
    assert np.abs(f["frame_embeds"][:4].numpy() - golden_flow["frame_embeds_first4"]).max() < 2e-5


def _missing_kp_main(rank, ws, port, paths, ckpt, kp_dir, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from vge import dist as VD
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        VD.run_eval_distributed(paths["generated_meshes"], paths["real"], ckpt, kp_dir, paths["real_kp"],
                                out_json=None, device="cuda:0")
        q.put((rank, "ok"))
    except VD.PeerRankFailed as e:
        q.put((rank, f"peer:{e}"))
    except FileNotFoundError as e:
        q.put((rank, f"own:{e}"))
    finally:
        dist.destroy_process_group()


def test_missing_keypoints_on_one_rank_stop_every_rank(golden_dataset, tmp_path):
    """The last generated video (rank 1's shard) has no keypoints.npy: rank 1 raises FileNotFoundError
    (utils.py:416-417) and rank 0 raises PeerRankFailed at the same exchange; neither waits in a collective."""
    import shutil
    paths, ckpt = golden_dataset
    kp = tmp_path / "generated_kps"
    shutil.copytree(paths["generated_kps"], kp)
    victim = sorted(d for d in kp.iterdir() if d.is_dir())[-1]
    (victim / "keypoints.npy").unlink()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_missing_kp_main, args=(r, 2, port, paths, ckpt, str(kp), q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = dict(q.get() for _ in range(2))
    assert got[1].startswith("own:") and "Expected keypoints" in got[1], got
    assert got[0].startswith("peer:"), got
