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


@pytest.mark.parametrize("overlap", ["1", "0"])
def test_two_rank_run_eval_matches_golden(golden_dataset, golden_meta, tmp_path, overlap):
    """Both phase orders: background generated-set decode + checkpoint read (default) and eval.py's serial order."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    paths, ckpt = golden_dataset
    out = str(tmp_path / "video_scores.json")
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, paths, ckpt, out, q, overlap)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = dict((r, res) for r, res, _ in (q.get(), q.get()))
    assert got[1] is None
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
