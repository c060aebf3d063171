"""world_size-2 gloo (CPU) tests of the multi-GPU composition in vge/dist.py.

The per-rank compute here is the oracle (the CPU restatement of eval.py); what is under test is the part
the GPU path shares verbatim: contiguous sharding of the sorted video lists, the deterministic all-gather +
rank-ordered sum of the stats / centroid sufficient statistics, and the gather of per-video scores to rank
0.  The merged result must equal the single-process reference golden vectors.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_bounds_partition():
    from vge.dist import shard_bounds
    for ws in range(1, 9):
        for n in range(0, 41):
            spans = [shard_bounds(n, r, ws) for r in range(ws)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def _rank_main(rank, ws, port, paths, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    import torch.distributed as dist
    import torch.nn.functional as F
    from oracle import evalflow as EF
    from oracle.encoder import OracleEncoder
    from oracle.featurize import RAW_ORDER, StatsAccumulator
    from vge import dist as VD
    from vge import synth
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        real = EF.scan_real(paths["real"])
        train = EF.split(real)
        mine = VD.shard(train, rank, ws)
        # ModalityStats: float64 sums / squares + frame counts, one all-gather, rank-ordered sum
        acc = StatsAccumulator()
        for cls, name, path, T in mine:
            pose, gori, betas, vit, kp = EF.load(path, paths["real_kp"], cls, require_kp=False)
            acc.add_video(pose, gori, betas, vit, kp)
        keys = [(k, m) for m in RAW_ORDER for k in ("raw", "diff")]
        dims = {}
        for cls, name, path, T in train[:1]:
            pose, gori, betas, vit, kp = EF.load(path, paths["real_kp"], cls, require_kp=False)
            probe = StatsAccumulator()
            probe.add_video(pose, gori, betas, vit, kp)
            dims = {k: probe.s[k].shape[0] for k in keys}
        flat_s = np.concatenate([acc.s.get(k, np.zeros(dims[k])) for k in keys] +
                                [acc.ss.get(k, np.zeros(dims[k])) for k in keys])
        n = np.array([acc.n.get(k, 0) for k in keys], np.int64)
        S, N = VD.stats_reduce_fn(torch.from_numpy(flat_s), n)
        S = S.numpy()
        off = 0
        tot = StatsAccumulator()
        for k in keys:
            tot.s[k] = S[off:off + dims[k]]
            off += dims[k]
        for k in keys:
            tot.ss[k] = S[off:off + dims[k]]
            off += dims[k]
        for k, c in zip(keys, N):
            tot.n[k] = int(c)
        stats = tot.finalize()
        mean, std = stats.concat()
        # centroids: f32 sums [C,256] + counts [C], one all-gather, rank-ordered sum
        sd = synth.make_state_dict(synth.DIMS_RAW, synth.DIMS_DIFF)
        enc = OracleEncoder(sd, synth.DIMS_RAW, synth.DIMS_DIFF)
        label_dict = {c: i for i, c in enumerate(sorted(real.keys()))}
        samples = [(cls, name, path, s) for cls, name, path, T in mine if T > 0 for s in EF.windows_for(T)]
        sums = torch.zeros(len(label_dict), 256)
        counts = torch.zeros(len(label_dict))
        if samples:
            seq, _, clss, _ = EF.encode_samples(enc, samples, paths["real_kp"], stats, batch_size=64)
            y = torch.as_tensor([label_dict[c] for c in clss], dtype=torch.long)
            sums.index_add_(0, y, seq)
            counts.index_add_(0, y, torch.ones_like(y, dtype=torch.float32))
        sums, counts = VD.centroid_reduce_fn(sums, counts)
        cents = F.normalize(sums / counts.clamp_min(1.0).unsqueeze(1), dim=-1)
        # scoring: this rank's contiguous block of the sorted generated list, no collective
        gen = sorted(EF.scan_generated(paths["generated_meshes"]), key=lambda it: it[2])
        gmine = VD.shard(gen, rank, ws)
        gs = [(cls, name, path, s) for cls, name, path, T in gmine for s in EF.windows_for(T)]
        combined = {}
        if gs:
            seq, fe, clss, names = EF.encode_samples(enc, gs, paths["generated_kps"], stats)
            ac = EF.ac_scores(seq, clss, names, cents, label_dict)
            tc = EF.tc_scores(fe, names)
            for v in sorted(set(ac) | set(tc)):
                combined[v] = {**({"ac": ac[v]} if v in ac else {}), **({"tc": tc[v]} if v in tc else {})}
        parts = VD.gather_to_rank0(combined)
        if rank == 0:
            q.put({"mean": mean, "std": std, "centroids": cents.numpy(), "counts": counts.numpy(),
                   "scores": VD.merge_scores(parts), "n_parts": len(parts), "sizes": [len(p) for p in parts]})
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ws", [2, 8])
def test_two_rank_gloo_flow_matches_single_process_golden(golden_dataset, golden_flow, golden_meta, ws):
    """World sizes 2 and 8 (config 4's one rank per GPU of an 8-GPU node, rehearsed on gloo): the same merged stats,
    centroids and scores as the single-process reference, every rank scoring its own contiguous shard."""
    paths, _ = golden_dataset
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, ws, port, paths, q)) for r in range(ws)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    out = q.get()
    assert out["n_parts"] == ws and min(out["sizes"]) > 0         # every rank scored videos
    np.testing.assert_allclose(out["mean"], golden_flow["stats_mean"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(out["std"], golden_flow["stats_std"], rtol=1e-6, atol=1e-7)
    assert np.array_equal(out["counts"], golden_flow["counts"])
    assert np.abs(out["centroids"] - golden_flow["centroids"]).max() < 2e-5
    ref = golden_meta["video_scores"]
    assert sorted(out["scores"]) == sorted(ref)
    worst = max(abs(ref[v][k] - out["scores"][v][k]) for v in ref for k in ref[v])
    assert worst < 1e-4, worst


def test_collective_device_policy(monkeypatch):
    """An nccl (RCCL) process group serves cuda tensors only: host tensors handed to the flow's exchanges (the
    int64 frame counts of the stats, the status flags of agree()) are staged on the rank's GPU; gloo keeps host
    tensors; device tensors stay where they are."""
    import torch.distributed as dist
    from vge import dist as VD
    monkeypatch.setattr(VD, "_rank_device", lambda: torch.device("cuda", 3))
    monkeypatch.setattr(dist, "get_backend", lambda *a, **k: "nccl")
    assert VD._collective_device(torch.zeros(2, dtype=torch.int64)) == torch.device("cuda", 3)
    meta = torch.zeros(2, device="meta")
    assert VD._collective_device(meta) == torch.device("cuda", 3)  # anything not cuda is staged
    monkeypatch.setattr(dist, "get_backend", lambda *a, **k: "gloo")
    assert VD._collective_device(torch.zeros(2)) == torch.device("cpu")


def test_flow_exchanges_stage_host_tensors_for_nccl(monkeypatch):
    """Every tensor stats_reduce_fn / centroid_reduce_fn / agree hand to all_gather under an nccl group is on the
    rank's device (a stand-in device here: the test host has no GPU), including the host int64 counts."""
    import torch.distributed as dist
    from vge import dist as VD
    seen = []

    class Staged(torch.Tensor):
        pass

    def fake_to(t, dev):
        assert dev == torch.device("cuda", 0), dev
        return t.clone().as_subclass(Staged)

    def fake_all_gather(parts, src):
        seen.append(isinstance(src, Staged))
        for p in parts:
            p.copy_(src)

    monkeypatch.setattr(VD, "in_group", lambda: True)
    monkeypatch.setattr(VD, "world", lambda: (0, 2))
    monkeypatch.setattr(dist, "get_backend", lambda *a, **k: "nccl")
    monkeypatch.setattr(dist, "all_gather", fake_all_gather)
    monkeypatch.setattr(VD, "_rank_device", lambda: torch.device("cuda", 0))
    orig_to = torch.Tensor.to

    def to(self, *a, **k):
        if a and isinstance(a[0], torch.device) and a[0].type == "cuda":
            return fake_to(self, a[0])
        return orig_to(self, *a, **k)

    monkeypatch.setattr(torch.Tensor, "to", to)
    s, c = VD.stats_reduce_fn(torch.ones(2, 5, dtype=torch.float64), np.array([3, 4], np.int64))
    assert s.dtype == torch.float64 and float(s.sum()) == 20.0 and c.tolist() == [6, 8]
    cs, cc = VD.centroid_reduce_fn(torch.ones(3, 256), torch.ones(3))
    assert float(cc.sum()) == 6.0
    VD.agree(None, "test")
    assert len(seen) == 5 and all(seen), seen


def _agree_main(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from vge import dist as VD
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        def phase():
            if rank == 1:
                raise FileNotFoundError("Expected keypoints at /nowhere/keypoints.npy")
            return rank
        try:
            VD.guarded("generated-set scoring", phase)
            q.put((rank, "ok"))
        except VD.PeerRankFailed as e:
            q.put((rank, f"peer:{e}"))
        except FileNotFoundError as e:
            q.put((rank, f"own:{e}"))
    finally:
        dist.destroy_process_group()


def test_error_on_one_rank_raises_on_every_rank():
    """A bad file seen by one rank only (its shard) makes every rank raise before the next exchange, instead of
    leaving the peers blocked in a collective until the backend timeout."""
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_agree_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = dict(q.get() for _ in range(2))
    assert got[1].startswith("own:") and "Expected keypoints" in got[1]
    assert got[0].startswith("peer:") and "[1]" in got[0]


def _digest_main(rank, ws, port, tmp, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from vge import dist as VD
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        gen = os.path.join(tmp, "gen")
        os.makedirs(gen, exist_ok=True)
        ckpt = os.path.join(tmp, "model.pt")
        if rank == 0:
            open(ckpt + ".r0", "wb").write(b"x" * 64)
        model = ckpt + ".r0" if rank == 0 else os.path.join(tmp, "missing.pt")  # rank 1 cannot read its checkpoint
        try:
            VD.run_eval_distributed(gen, os.path.join(tmp, "real"), model, None, None, out_json=None, device="cpu",
                                    stats_cache=os.path.join(tmp, "stats.npz"))
            q.put((rank, "ok"))
        except VD.PeerRankFailed as e:
            q.put((rank, f"peer:{e}"))
        except OSError as e:
            q.put((rank, f"own:{type(e).__name__}"))
    finally:
        dist.destroy_process_group()


def test_unreadable_checkpoint_for_the_stats_cache_stops_every_rank(tmp_path):
    """The stats-cache fingerprint reads the checkpoint before the first collective: a rank that cannot read it
    raises, and its peer raises PeerRankFailed instead of waiting in the cache-hit all-gather."""
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_digest_main, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = dict(q.get() for _ in range(2))
    assert got[1] == "own:FileNotFoundError", got
    assert got[0].startswith("peer:") and "[1]" in got[0], got
