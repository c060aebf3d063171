"""The real set's stats + centroid artifact (vge/stats_cache.py; SURVEY.md 7 hard part 4, 8(e) option 2).

CPU: the file round trip, fingerprint misses (a real file touched, another checkpoint / compute mode / stride), the
shape checks, and the all-ranks agreement on a hit (gloo, world size 2).  GPU: scores read from the artifact equal a
fresh run's bit for bit, in one process and on two ranks, and the cached runs skip the real set."""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from vge import stats_cache as SC
from vge.data import VideoItem


def _items(tmp_path, n=3):
    items = []
    for k in range(n):
        p = tmp_path / f"v{k}.npz"
        p.write_bytes(b"x" * (10 + k))
        items.append(VideoItem(cls="Run", name=p.name, path=str(p), length=32, vit_dim=1024))
    return items


def _arrays(C=4):
    rng = np.random.default_rng(0)
    return (rng.normal(size=(2, 2596)), np.array([320, 300], np.int64), rng.normal(size=(C, 256)).astype(np.float32),
            np.arange(1, C + 1, dtype=np.float32))


def test_round_trip_and_misses(tmp_path):
    items = _items(tmp_path)
    fp = SC.fingerprint(items, None, "ab" * 32, "f32x3", 32, 8)
    path = str(tmp_path / "stats.npz")
    ss, sc, cs, cc = _arrays()
    SC.save(path, fp, ss, sc, cs, cc, ["A", "B", "C", "D"])
    got = SC.load(path, fp)
    assert got is not None and got["classes"] == ["A", "B", "C", "D"]
    for k, v in (("stats_sums", ss), ("stats_counts", sc), ("cent_sums", cs), ("cent_counts", cc)):
        assert got[k].dtype == np.asarray(v).dtype and np.array_equal(got[k], v), k
    assert SC.load(path, SC.fingerprint(items, None, "cd" * 32, "f32x3", 32, 8)) is None   # another checkpoint
    assert SC.load(path, SC.fingerprint(items, None, "ab" * 32, "f16", 32, 8)) is None     # another compute mode
    assert SC.load(path, SC.fingerprint(items, None, "ab" * 32, "f32x3", 32, 16)) is None  # another stride
    assert SC.load(path, SC.fingerprint(items[:2], None, "ab" * 32, "f32x3", 32, 8)) is None
    os.utime(items[1].path, ns=(1, 1))                                                      # a real file changed
    assert SC.load(path, SC.fingerprint(items, None, "ab" * 32, "f32x3", 32, 8)) is None
    assert SC.load(str(tmp_path / "absent.npz"), fp) is None
    (tmp_path / "junk.npz").write_bytes(b"not an npz")
    assert SC.load(str(tmp_path / "junk.npz"), fp) is None
    whole = open(path, "rb").read()                                                         # a partial copy
    for cut in (len(whole) // 2, len(whole) - 30, 100):
        (tmp_path / "cut.npz").write_bytes(whole[:cut])
        assert SC.load(str(tmp_path / "cut.npz"), fp) is None


def test_kernel_switches_are_in_the_fingerprint(tmp_path, monkeypatch):
    """A cache written under one kernel selection / numerics switch (VGE_F16_MIX, VGE_X3S, ...) is a miss under
    another; the library version is recorded too."""
    items = _items(tmp_path)
    monkeypatch.delenv("VGE_F16_MIX", raising=False)
    fp = SC.fingerprint(items, None, "ab" * 32, "f16", 32, 8)
    assert "version" in fp["kernels"] and fp["kernels"]["env"]["VGE_F16_MIX"] is None
    path = str(tmp_path / "stats.npz")
    SC.save(path, fp, *_arrays(), ["A", "B", "C", "D"])
    assert SC.load(path, SC.fingerprint(items, None, "ab" * 32, "f16", 32, 8)) is not None
    monkeypatch.setenv("VGE_F16_MIX", "0")
    assert SC.load(path, SC.fingerprint(items, None, "ab" * 32, "f16", 32, 8)) is None


def test_shape_mismatch_is_a_miss(tmp_path):
    items = _items(tmp_path)
    fp = SC.fingerprint(items, None, "ab" * 32, "f32x3", 32, 8)
    ss, sc, cs, cc = _arrays()
    path = str(tmp_path / "stats.npz")
    SC.save(path, fp, ss, sc, cs, cc, ["A", "B", "C"])  # 3 classes for 4 centroid rows
    assert SC.load(path, fp) is None


def test_model_digest_of_state_dict_and_file(tmp_path):
    sd = {"b": np.ones((2, 3), np.float32), "a": np.zeros(4, np.float32)}
    d1 = SC.model_digest(sd)
    assert d1 == SC.model_digest(dict(reversed(list(sd.items()))))  # key order does not matter
    sd2 = dict(sd, a=np.full(4, 1e-7, np.float32))
    assert SC.model_digest(sd2) != d1
    f = tmp_path / "ck.pt"
    f.write_bytes(b"checkpoint bytes")
    assert SC.model_digest(str(f)) == SC.model_digest(str(f)) != SC.model_digest(sd)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _agree_main(rank, ws, port, flags, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from vge import dist as VD
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        q.put((rank, [VD.all_agree(f[rank]) for f in flags]))
    finally:
        dist.destroy_process_group()


def test_cache_hit_needs_every_rank():
    """A hit on one rank and a miss on another must send both ranks down the full flow (else one would wait in the
    stats exchange forever)."""
    flags = [(True, True), (True, False), (False, True), (False, False)]
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_agree_main, args=(r, 2, port, flags, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs)
    got = dict(q.get() for _ in range(2))
    assert got[0] == got[1] == [True, False, False, False]


@pytest.mark.gpu
def test_cached_scores_equal_fresh_run_bit_for_bit(golden_dataset, golden_meta, tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vge import eval as VE
    paths, ckpt = golden_dataset
    args = (paths["generated_meshes"], paths["real"], ckpt, paths["generated_kps"], paths["real_kp"])
    cache = str(tmp_path / "stats.npz")
    fresh_t, miss_t, hit_t = {}, {}, {}
    fresh = VE.run_eval(*args, out_json=None, timings=fresh_t)
    miss = VE.run_eval(*args, out_json=None, timings=miss_t, stats_cache=cache)
    hit = VE.run_eval(*args, out_json=None, timings=hit_t, stats_cache=cache)
    assert (fresh_t["stats_cache"], miss_t["stats_cache"], hit_t["stats_cache"]) == ("off", "miss", "hit")
    assert json.dumps(fresh, sort_keys=True) == json.dumps(miss, sort_keys=True) == json.dumps(hit, sort_keys=True)
    ref = golden_meta["video_scores"]
    assert max(abs(ref[v][k] - hit[v][k]) for v in ref for k in ref[v]) < 1e-4
    print(f"setup (stats + centroids) s: fresh {fresh_t['stats_s'] + fresh_t['centroids_s']:.3f}, cached "
          f"{hit_t['stats_s'] + hit_t['centroids_s']:.3f}")
    # another compute mode is a miss (its centroids differ)
    t = {}
    VE.run_eval(*args, out_json=None, timings=t, stats_cache=cache, compute="f16")
    assert t["stats_cache"] == "miss"


def _rank_main(rank, ws, port, paths, ckpt, cache, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from vge import dist as VD
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        out = []
        for c in (None, cache, cache):  # fresh, miss (rank 0 writes), hit
            t = {}
            dist.barrier()
            res = VD.run_eval_distributed(paths["generated_meshes"], paths["real"], ckpt, paths["generated_kps"],
                                          paths["real_kp"], out_json=None, device="cuda:0", timings=t, stats_cache=c)
            out.append((res, t["stats_cache"]))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_two_rank_cached_flow_equals_fresh(golden_dataset, tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    paths, ckpt = golden_dataset
    cache = str(tmp_path / "stats.npz")
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, paths, ckpt, cache, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = dict(q.get() for _ in range(2))
    assert [s for _, s in got[0]] == [s for _, s in got[1]] == ["off", "miss", "hit"]
    fresh, miss, hit = (r for r, _ in got[0])
    assert json.dumps(fresh, sort_keys=True) == json.dumps(miss, sort_keys=True) == json.dumps(hit, sort_keys=True)
