"""The TokenHMR front end (mesh_generator.py:101-145): single-person gate and ViTDetDataset's crop.

The crop geometry and warp are third-party (4D-Humans ViTDetDataset / generate_image_patch_cv2, cv2.warpAffine,
skimage.filters.gaussian) restated in oracle/hmr.py; the detector is detectron2's Faster R-CNN in the reference and
the YOLOX-L of vge.dwpose here (stand-in): parity UNPINNED.  Checked:
  CPU   the gate rule (exactly one box > 0.5 among the first two NMS-kept persons, >= 80 % of the frames) and the
        crop geometry (center, 2.5x scale, 192:256 aspect expansion, blur trigger) on hand-computed boxes
  GPU   vge_hmr_crop vs oracle.vitdet_crop: every byte equal on the unblurred path (float bilinear without
        contraction on both sides), within 1 where the anti-alias Gaussian applies; boxes partly outside the frame
        (border 0); the full front end (YOLOX detect -> gate -> crops) against the oracle's gate and crops on the
        detector's own boxes and scores
"""
import numpy as np
import pytest
import torch

DEV = "cuda:0"
gpu = pytest.mark.gpu


def test_single_person_gate_rule():
    from oracle.hmr import single_person_mask as oracle_mask
    from vge.extract import SINGLE_PERSON_MIN_FRACTION, single_person_mask
    s = np.array([[0.9, 0.0], [0.9, 0.6], [0.4, 0.0], [0.51, 0.5], [0.0, 0.0], [0.5, 0.2]], np.float32)
    want = np.array([True, False, False, True, False, False])
    assert np.array_equal(single_person_mask(s), want)
    assert np.array_equal(oracle_mask(s), want)
    assert SINGLE_PERSON_MIN_FRACTION == 0.8


def test_vitdet_geometry_by_hand():
    from oracle.hmr import expand_to_aspect_ratio, vitdet_geometry
    # 40 x 100 box: scale * 200 = (100, 250); h/w = 2.5 >= 256/192 -> w_new = 250 * 0.75 = 187.5; bbox = 250
    cx, cy, k, sigma = vitdet_geometry([10, 20, 50, 120])
    assert (cx, cy) == (30.0, 70.0) and abs(float(k) - 250 / 256) < 1e-7 and sigma == 0.0
    assert np.allclose(expand_to_aspect_ratio((100, 250)), (187.5, 250))
    # 200 x 100 box: (500, 250) -> h_new = max(500 * 4/3, 250) = 666.67; downsampling 666.67 / 512 = 1.30 > 1.1
    cx, cy, k, sigma = vitdet_geometry([0, 0, 200, 100])
    assert abs(float(k) * 256 - 2000 / 3) < 1e-3 and abs(sigma - (2000 / 3 / 512 - 1) / 2) < 1e-9


@gpu
@pytest.mark.parametrize("size,boxes", [
    (256, [[60, 40, 140, 230], [0, 0, 256, 256], [-30, 100, 80, 300], [120.5, 10.25, 131.75, 40.5]]),
    (512, [[10, 10, 500, 480], [200, 100, 320, 450], [0, 0, 512, 300]]),
    (256, [[-400, -400, 660, 660], [-60, -300, 300, 560]]),  # radii 12 (> the old cap of 8) and 6
])
def test_crop_matches_oracle(size, boxes):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle.hmr import vitdet_crop, vitdet_geometry
    from vge import synth
    from vge.hmr import crop_persons
    frames = synth.make_frames(31 + size, 2, size, size)
    fo = np.arange(len(boxes)) % 2
    got = crop_persons(torch.from_numpy(frames).to(DEV), np.asarray(boxes, np.float32), fo).cpu().numpy()
    for i, b in enumerate(boxes):
        ref = vitdet_crop(frames[fo[i]], b)
        d = np.abs(got[i].astype(np.int32) - ref.astype(np.int32)).max()
        blurred = vitdet_geometry(b)[3] > 0
        assert d <= (1 if blurred else 0), (i, b, d, blurred)
    with pytest.raises(Exception, match="box"):
        crop_persons(torch.from_numpy(frames).to(DEV), np.array([[10, 10, 10, 50]], np.float32))
    with pytest.raises(Exception, match="too large"):  # radius 44 > 32: refused, not truncated
        crop_persons(torch.from_numpy(frames).to(DEV), np.array([[-1500, -1500, 2000, 2000]], np.float32))


@gpu
def test_front_end_detect_gate_crop():
    """YOLOX (small random-weight config) on full frames -> scores -> gate -> crops of the kept frames, against the
    oracle gate and crop on the detector's own boxes (the detector network itself is checked in test_yolox.py)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle.hmr import single_person_mask as oracle_mask
    from oracle.hmr import vitdet_crop
    from vge import synth
    from vge.dwpose import YoloxConfig, YoloxDetector
    from vge.extract import tokenhmr_front
    cfg = YoloxConfig(in_size=128, width=16, depth=1, head_ch=64)
    det = YoloxDetector(synth.make_yolox_state_dict(cfg, gain=2.0), cfg, device=DEV, chunk=8)
    frames = synth.make_frames(5, 10, 256, 256)
    fr = torch.from_numpy(frames).to(DEV)
    boxes, npers, scores = det.detect(fr, with_scores=True)
    b, s = boxes.cpu().numpy(), scores.cpu().numpy()
    n = npers.cpu().numpy()
    assert np.array_equal(n, (s[:, 0] > 0).astype(np.int32) + (s[:, 1] > 0))  # scores sit beside the kept persons
    # force a deterministic mix of gate outcomes on the detector's own boxes
    s2 = s.copy()
    s2[:, 0] = np.where(np.arange(10) == 9, 0.2, 0.9)   # frame 9: nobody above 0.5
    s2[:, 1] = np.where(np.arange(10) == 3, 0.7, 0.1)   # frame 3: two people above 0.5
    b2 = b.copy()
    b2[:, 0] = [[20 + i, 30, 120 + 5 * i, 230] for i in range(10)]
    keep_ref = np.flatnonzero(oracle_mask(s2))
    out = tokenhmr_front(det, fr, detections=(b2, n, s2))
    assert out is not None
    idx, crops = out
    assert np.array_equal(idx, keep_ref) and len(idx) == 8
    c = crops.cpu().numpy()
    for j, f in enumerate(idx):
        assert np.array_equal(c[j], vitdet_crop(frames[f], b2[f, 0]))
    s3 = s2.copy()
    s3[:1, 0] = 0.1                                    # one more frame fails: 7 / 10 < 80 % -> rejected
    assert tokenhmr_front(det, fr, detections=(b2, n, s3)) is None
