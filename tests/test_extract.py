"""Extraction drivers (vge/extract.py): the per-video npz format is pinned by a file the reference's own
save_video_npz wrote (tests/golden/make_npz_format_golden.py); the single-person gate restates
mesh_generator.py:101-117; the GPU test runs TokenHMR + DWPose into files the scorer's reader loads back."""
import json

import numpy as np
import pytest
import torch

from tests.conftest import GOLDEN

DEV = "cuda:0"


def _sample_mesh_info():
    from tests.golden.make_npz_format_golden import sample_mesh_info
    return sample_mesh_info()


def test_save_video_npz_matches_reference_file(tmp_path):
    from vge.extract import save_video_npz
    p = save_video_npz("Action/v_ref", _sample_mesh_info(), out_root=tmp_path,
                       meta={"action": "Action", "video": "v_ref.avi", "source_path": "x/v_ref.avi"})
    assert p == str(tmp_path / "Action" / "v_ref.npz")
    ref = np.load(GOLDEN / "npz_format" / "Action" / "v_ref.npz")
    got = np.load(p)
    assert sorted(ref.files) == sorted(got.files)
    for k in ref.files:
        assert ref[k].dtype == got[k].dtype and ref[k].shape == got[k].shape, k
        np.testing.assert_array_equal(ref[k], got[k], err_msg=k)
    assert json.loads(str(got["meta"]))["video"] == "v_ref.avi"
    np.testing.assert_array_equal(got["frame_idx"], [0, 2, 4, 7])


def test_reference_npz_reads_through_the_scorer_loader():
    from vge.data import VideoItem, load_clip
    path = str(GOLDEN / "npz_format" / "Action" / "v_ref.npz")
    clip = load_clip(VideoItem(cls="Action", name="v_ref.npz", path=path, length=4, vit_dim=16), None, False)
    assert clip["pose"].shape == (4, 23, 3, 3) and clip["global_orient"].shape == (4, 1, 3, 3)
    assert clip["betas"].shape == (4, 10) and clip["vit"].shape == (4, 16)


def test_single_person_gate():
    from vge.extract import single_person_frames
    np.testing.assert_array_equal(single_person_frames([1, 1, 1, 1, 0]), [0, 1, 2, 3])   # 4/5 = 0.8: kept
    assert single_person_frames([1, 1, 1, 0, 2]) is None                                 # 3/5 < 0.8
    assert single_person_frames([0, 0]) is None and single_person_frames([]) is None
    np.testing.assert_array_equal(single_person_frames([1] * 9 + [3]), np.arange(9))


@pytest.mark.gpu
def test_gate_videos_compacts_kept_frames():
    """vge.extract.gate_videos (the e2e bench's per-pass gate): accepted videos, their kept frames and frame-store
    descriptors, video by video the same decision as single_person_frames (mesh_generator.py:101-117)."""
    from vge.extract import gate_videos, single_person_frames
    T = 10
    rng = np.random.default_rng(3)
    keep = np.ones(5 * T, bool)
    keep[T + 2] = keep[T + 7] = False                    # video 1: 8 / 10 kept (accepted)
    keep[2 * T:2 * T + 3] = False                        # video 2: 7 / 10 (rejected)
    keep[3 * T:4 * T] = False                            # video 3: none (rejected)
    keep[4 * T + 9] = False                              # video 4: 9 / 10
    acc, kept, desc = gate_videos(keep, T, frame_off=100)
    assert acc.tolist() == [0, 1, 4]
    want = [v * T + f for v in (0, 1, 4) for f in single_person_frames(np.where(keep[v * T:(v + 1) * T], 1, 0))]
    assert kept.tolist() == want
    assert desc.tolist() == [[100, 10, 0, T], [110, 8, T, T], [118, 9, 4 * T, T]]
    # every decision matches the per-video rule on random masks
    for _ in range(20):
        k = rng.random(6 * T) < 0.85
        acc, kept, desc = gate_videos(k, T)
        ref = [v for v in range(6) if single_person_frames(np.where(k[v * T:(v + 1) * T], 1, 0)) is not None]
        assert acc.tolist() == ref and int(desc[:, 1].sum()) == kept.size


def test_extract_video_round_trip(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vge import dwpose as D, hmr as H, synth
    from vge.data import VideoItem, load_clip
    from vge.extract import extract_video
    hcfg = H.HmrConfig(embed_dim=256, depth=1, heads=4, mlp_dim=256, dec_dim=256, dec_depth=1, dec_heads=4,
                       dec_mlp=256, tok_num=4, tok_classes=256, tok_code_dim=256)
    hmr = H.HmrExtractor(synth.make_hmr_state_dict(hcfg), hcfg, device=DEV, max_frames=8)
    ycfg = D.YoloxConfig(in_size=128, width=16, depth=1, head_ch=64)
    pcfg = D.RtmposeConfig(in_h=128, in_w=96, stem_ch=16, stage_ch=(32, 64, 128, 256), stage_blocks=(1, 1, 1, 1))
    wb = D.Wholebody(D.YoloxDetector(synth.make_yolox_state_dict(ycfg), ycfg, device=DEV, chunk=8),
                     D.DwposeExtractor(synth.make_rtmpose_state_dict(pcfg), pcfg, device=DEV, max_instances=16))
    frames = torch.from_numpy(synth.make_frames(5, 6)).to(DEV)
    counts = [1, 1, 2, 1, 1, 1]                                  # frame 2 fails the single-person gate
    paths = extract_video(hmr, wb, frames, frames, "Soccer", "v_x_01.avi", tmp_path / "meshes", tmp_path / "kps",
                          person_counts=counts)
    z = np.load(paths["npz"])
    np.testing.assert_array_equal(z["frame_idx"], [0, 1, 3, 4, 5])
    ref = hmr.extract(frames[torch.tensor([0, 1, 3, 4, 5], device=DEV)])
    np.testing.assert_array_equal(z["vit"], ref["vit"].cpu().numpy())
    clip = load_clip(VideoItem(cls="Soccer", name="v_x_01.npz", path=paths["npz"], length=5, vit_dim=256),
                     str(tmp_path / "kps"), True)
    assert clip["keypoints"].shape == (6, 120)
    np.testing.assert_array_equal(clip["keypoints"], wb(frames).cpu().numpy())
    assert extract_video(hmr, wb, frames, frames, "Soccer", "v_x_02.avi", tmp_path / "meshes", tmp_path / "kps",
                         person_counts=[2, 2, 1, 0, 1, 1])["npz"] is None  # 3/6 single-person frames: rejected
