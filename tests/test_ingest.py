"""Native on-disk ingest (include/vge_ingest.h, vge/ingest.py) against the
reference's own reader, np.load (utils.py:383-424), as the checker: bit-identical frame stores on the
golden dataset and on synthetic files covering savez / savez_compressed members, float64 arrays,
keypoint files shorter than the mesh, absent and unreadable keypoint files, empty and truncated npz, and
the packed sidecar round trip.  CPU only (host code in libvge.so)."""
import os
from pathlib import Path

import numpy as np
import pytest

from vge import ingest, synth
from vge.data import VideoItem, create_dataset_from_generated_meshes, load_clip, pack_frame_store


def numpy_store(items, kp_dir, require_kp):
    clips = [load_clip(it, kp_dir, require_kp) for it in items]
    return pack_frame_store(clips, [it.name for it in items], [it.cls for it in items])


def assert_same(a, b):
    assert a.names == b.names and a.classes == b.classes
    assert np.array_equal(a.videos, b.videos)
    for k in ("pose", "gori", "betas", "vit"):
        assert getattr(a, k).shape == getattr(b, k).shape, k
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
    nk = int(a.videos[:, 3].sum()) if len(a.videos) else 0
    assert np.array_equal(a.kp[:nk], b.kp[:nk])


def _write(root: Path, name, T, kp_len=None, compressed=True, f64=False, kp=True, vit_dim=64, seed=0):
    c = synth.make_clip(synth.SEED_GEN, seed, max(T, 1), kp_len=kp_len, vit_dim=vit_dim)
    arrs = dict(pose=c.pose[:T], global_orient=c.global_orient[:T], betas=c.betas[:T], vit=c.vit[:T])
    if f64:
        arrs = {k: v.astype(np.float64) for k, v in arrs.items()}
    path = root / "gen" / f"{name}.npz"
    path.parent.mkdir(parents=True, exist_ok=True)
    (np.savez_compressed if compressed else np.savez)(path, **arrs, frame_idx=np.arange(T, dtype=np.int32))
    if kp:
        kp_path = root / "generated_kps" / name / "keypoints.npy"
        kp_path.parent.mkdir(parents=True, exist_ok=True)
        np.save(kp_path, c.keypoints.astype(np.float64) if f64 else c.keypoints)
    return VideoItem(cls="Unknown", name=path.name, path=str(path), length=T, vit_dim=vit_dim)


def test_golden_dataset_matches_numpy_reader(golden_dataset):
    paths, _ = golden_dataset
    gen = create_dataset_from_generated_meshes(paths["generated_meshes"]).items
    a = ingest.load_frame_store_native(gen, paths["generated_kps"], require_kp=True, threads=4)
    assert_same(a, numpy_store(gen, paths["generated_kps"], True))
    from vge.data import NpzVideoDataset
    real = NpzVideoDataset(paths["real"]).items
    a = ingest.load_frame_store_native(real, paths["real_kp"], require_kp=False, threads=3)
    assert_same(a, numpy_store(real, paths["real_kp"], False))


def test_formats_and_edge_cases(tmp_path):
    kp_dir = str(tmp_path / "generated_kps")
    items = [_write(tmp_path, "a", 32), _write(tmp_path, "b", 64, kp_len=50, seed=1),
             _write(tmp_path, "c", 5, compressed=False, seed=2), _write(tmp_path, "d", 40, f64=True, seed=3),
             _write(tmp_path, "e", 0, kp_len=0, seed=4), _write(tmp_path, "f", 33, kp=False, seed=5)]
    # without require_kp: "f" has no keypoints (kp_frames 0), like load_clip
    a = ingest.load_frame_store_native(items, kp_dir, require_kp=False, threads=2)
    assert_same(a, numpy_store(items, kp_dir, False))
    assert a.videos[5, 3] == 0 and a.videos[1, 3] == 50 and a.videos[4, 1] == 0
    # require_kp: the missing file raises like utils.py:416-417
    with pytest.raises(FileNotFoundError):
        ingest.load_frame_store_native(items, kp_dir, require_kp=True)
    a = ingest.load_frame_store_native(items[:5], kp_dir, require_kp=True, threads=1)
    assert_same(a, numpy_store(items[:5], kp_dir, True))
    # no keypoint dir at all
    a = ingest.load_frame_store_native(items, None, require_kp=False)
    assert_same(a, numpy_store(items, None, False))


def test_unreadable_files(tmp_path):
    kp_dir = str(tmp_path / "generated_kps")
    good = _write(tmp_path, "g", 32)
    bad = _write(tmp_path, "t", 32, seed=7)
    data = Path(bad.path).read_bytes()
    Path(bad.path).write_bytes(data[: len(data) // 2])  # truncated: no central directory
    with pytest.raises(RuntimeError):
        ingest.load_frame_store_native([good, bad], kp_dir, require_kp=False)
    junk = tmp_path / "junk.npz"
    junk.write_bytes(b"PK\x03\x04 not really a zip")
    with pytest.raises(RuntimeError):
        ingest.load_frame_store_native([VideoItem("Unknown", "junk.npz", str(junk), 1, 64)], None, False)
    # a keypoints.npy that is not [T', 120] float
    k = _write(tmp_path, "k", 32, seed=8)
    np.save(tmp_path / "generated_kps" / "k" / "keypoints.npy", np.zeros((32, 7), np.float32))
    with pytest.raises(RuntimeError):
        ingest.load_frame_store_native([k], kp_dir, require_kp=True)
    a = ingest.load_frame_store_native([good, k], kp_dir, require_kp=False)
    assert a.videos[1, 3] == 0 and a.videos[0, 3] == 32


def test_sidecar_round_trip(tmp_path):
    kp_dir = str(tmp_path / "generated_kps")
    items = [_write(tmp_path, f"s{i}", 32 + 8 * i, kp_len=30 + i, seed=10 + i) for i in range(5)]
    a = ingest.load_frame_store_native(items, kp_dir, require_kp=True)
    p = str(tmp_path / "store.vgefs")
    ingest.save_sidecar(a, p)
    b = ingest.load_sidecar(p, pinned=False)
    assert_same(a, b)
    assert os.path.getsize(p) % 4096 != 1  # written
    with open(p, "r+b") as f:
        f.write(b"XXXX")
    with pytest.raises(RuntimeError):
        ingest.load_sidecar(p, pinned=False)


def _zip64_with_wrapping_cd(src: bytes) -> bytes:
    """`src` (a valid npz) with a zip64 end record whose central-directory offset + size wrap around 2^64."""
    import struct
    e = src.rindex(b"PK\x05\x06")
    z64_off = e
    rec = struct.pack("<IQHHIIQQQQ", 0x06064B50, 44, 45, 45, 0, 0, 1, 1, 32, (1 << 64) - 16)
    loc = struct.pack("<IIQI", 0x07064B50, 0, z64_off, 1)
    eocd = bytearray(src[e:])
    eocd[10:12] = b"\xff\xff"
    eocd[12:16] = b"\xff\xff\xff\xff"
    eocd[16:20] = b"\xff\xff\xff\xff"
    return src[:e] + rec + loc + bytes(eocd)


def _patch_shape(raw: bytes, old: bytes, new: bytes) -> bytes:
    """Replace an npy header's shape text in place, keeping the header length (the padding absorbs it)."""
    i = raw.index(old)
    end = raw.index(b"\n", i)
    line = raw[i:end].replace(old, new, 1).rstrip(b" ")
    assert len(line) <= end - i
    return raw[:i] + line + b" " * (end - i - len(line)) + raw[end:]


def test_crafted_sizes_are_rejected_not_read(tmp_path):
    """Bounds checks on untrusted npz / npy input cannot wrap (zip64 offsets, npy shapes whose element count
    overflows): each file is refused with an error instead of being read out of bounds."""
    kp_dir = str(tmp_path / "generated_kps")
    z = _write(tmp_path, "z", 32, seed=20)
    Path(z.path).write_bytes(_zip64_with_wrapping_cd(Path(z.path).read_bytes()))
    with pytest.raises(RuntimeError):
        ingest.load_frame_store_native([z], kp_dir, require_kp=False)
    # keypoints.npy whose header claims 2^62 rows of 120 (count * itemsize overflows uint64)
    k = _write(tmp_path, "kk", 32, seed=21)
    kp_file = tmp_path / "generated_kps" / "kk" / "keypoints.npy"
    kp_file.write_bytes(_patch_shape(kp_file.read_bytes(), b"(32, 120)", f"({1 << 62}, 120)".encode()))
    with pytest.raises(RuntimeError):
        ingest.load_frame_store_native([k], kp_dir, require_kp=True)
    # an npz (stored members) whose pose member claims 2^40 frames
    p = tmp_path / "gen" / "big.npz"
    np.savez(p, pose=np.zeros((2, 23, 3, 3), np.float32), global_orient=np.zeros((2, 1, 3, 3), np.float32),
             betas=np.zeros((2, 10), np.float32), vit=np.zeros((2, 64), np.float32))
    p.write_bytes(_patch_shape(p.read_bytes(), b"(2, 23, 3, 3)", f"({1 << 40}, 23, 3, 3)".encode()))
    big = VideoItem("Unknown", "big.npz", str(p), 2, 64)
    with pytest.raises(RuntimeError):
        ingest.load_frame_store_native([big], None, require_kp=False)


def test_default_thread_count_ignores_torchrun_single_thread(monkeypatch):
    """torchrun exports OMP_NUM_THREADS=1 for nproc_per_node > 1; the decoder must still use the rank's CPU share."""
    from vge import lib as L
    lib = L.load()
    lib.vge_ingest_default_threads.restype = __import__("ctypes").c_int
    monkeypatch.setenv("VGE_INGEST_THREADS", "5")
    assert lib.vge_ingest_default_threads() == 5
    monkeypatch.delenv("VGE_INGEST_THREADS")
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    assert lib.vge_ingest_default_threads() == 3
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    share = lib.vge_ingest_default_threads()
    assert share == min(64, len(os.sched_getaffinity(0))) or share >= 1
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    assert lib.vge_ingest_default_threads() == max(1, share // 2)


def test_explicit_keypoint_layout(tmp_path):
    """keypoint_path: "auto" is the reference's name sniffing (utils.py:410-417); "flat" / "per_class" override
    it, so a flat keypoint dir with an arbitrary name resolves; the native and numpy readers agree under it."""
    from vge import data
    assert data.keypoint_path("/x/generated_kps", "PushUps", "v0") == "/x/generated_kps/v0/keypoints.npy"
    assert data.keypoint_path("/x/kps", "PushUps", "v0") == "/x/kps/PushUps/v0/keypoints.npy"
    assert data.keypoint_path("/x/kps", "PushUps", "v0", layout="flat") == "/x/kps/v0/keypoints.npy"
    assert data.keypoint_path("/x/SAVE_GEN", "PushUps", "v0", layout="per_class") == \
        "/x/SAVE_GEN/PushUps/v0/keypoints.npy"
    with pytest.raises(ValueError):
        data.keypoint_path("/x", "PushUps", "v0", layout="nested")
    with pytest.raises(ValueError):
        data.set_keypoint_layout("nested")

    mesh_dir, kp_dir = tmp_path / "meshes", tmp_path / "my_kps"
    mesh_dir.mkdir()
    items = []
    for i in range(2):
        c = synth.make_clip(synth.SEED_GEN, i, 33)
        p = mesh_dir / f"PushUps_{i}.npz"
        np.savez(p, pose=c.pose, global_orient=c.global_orient, betas=c.betas, vit=c.vit)
        (kp_dir / p.stem).mkdir(parents=True)
        np.save(kp_dir / p.stem / "keypoints.npy", c.keypoints)
        items.append(VideoItem(cls="PushUps", name=p.name, path=str(p), length=33, vit_dim=1024))
    try:
        data.set_keypoint_layout("flat", str(kp_dir) + "/")     # per directory (normalised path)
        assert data.get_keypoint_layout(str(kp_dir)) == "flat" and data.get_keypoint_layout("/other") == "auto"
        a = ingest.load_frame_store_native(items, str(kp_dir), require_kp=True)
        b = numpy_store(items, str(kp_dir), True)
        assert_same(a, b)
        assert int(a.videos[:, 3].sum()) == 66
        data.clear_keypoint_layouts()   # the reference's rule reads my_kps as per-class: keypoints absent
        with pytest.raises(Exception):
            numpy_store(items, str(kp_dir), True)
    finally:
        data.clear_keypoint_layouts()


def test_kp_layout_flag_needs_its_directory():
    from vge import eval as VE
    with pytest.raises(SystemExit):
        VE.main(["--generated-meshes", "g", "--real-meshes", "r", "--model", "m.pt", "--kp-layout", "flat"])


@pytest.mark.parametrize("flags", [["--keypoints", "k"], ["--real-keypoints", "rk"]])
def test_one_keypoint_dir_without_the_other_is_a_usage_error(flags):
    """Keypoints on one side only would featurise the generated set in a layout the real-set stats do not have; the
    reference raises in both cases (feature width / keypoints_raw_mean None), the CLI refuses it up front."""
    from vge import eval as VE
    with pytest.raises(SystemExit):
        VE.main(["--generated-meshes", "g", "--real-meshes", "r", "--model", "m.pt", *flags])


@pytest.mark.parametrize("kp_dir,stats_layout", [(None, "kp"), ("some/kps", "nokp")])
def test_feature_layout_must_match_the_stats(kp_dir, stats_layout):
    """extract_window_features refuses a generated keypoint dir whose layout differs from the stats' (run_eval and
    run_eval_distributed go through it) before anything is decoded or launched."""
    from types import SimpleNamespace
    from vge import eval as VE
    from vge.data import NpzVideoDataset
    stats = SimpleNamespace(layout=stats_layout)
    with pytest.raises(ValueError, match="feature layout"):
        VE.extract_window_features(None, NpzVideoDataset("", items=[]), kp_dir, stats, device="cpu")
