"""The TokenHMR front end (mesh_generator.py:101-145): single-person gate and ViTDetDataset's crop.

The crop geometry and warp are third-party (4D-Humans ViTDetDataset / generate_image_patch_cv2, cv2.warpAffine,
skimage.filters.gaussian) restated in oracle/hmr.py; the detector is detectron2's Faster R-CNN X101-32x8d-FPN
(vge.frcnn, checked stage by stage in test_frcnn.py): parity vs the upstream weights UNPINNED.  Checked:
  CPU   the gate rule (exactly one person instance > 0.5, >= 80 % of the frames) and the crop geometry (center, 2.5x
        scale, 192:256 aspect expansion, blur trigger) on hand-computed boxes
  GPU   vge_hmr_crop vs oracle.vitdet_crop: every byte equal on the unblurred path (float bilinear without
        contraction on both sides), within 1 where the anti-alias Gaussian applies; boxes partly outside the frame
        (border 0); the full front end (Faster R-CNN detect -> gate -> crops): the detector's person outputs agree
        with its instance list, and the gate / crops equal the oracle's on the detector's own boxes
"""
import numpy as np
import pytest
import torch

DEV = "cuda:0"
gpu = pytest.mark.gpu


def test_single_person_gate_rule():
    from vge.extract import SINGLE_PERSON_MIN_FRACTION, gate_mask, single_person_frames
    assert np.array_equal(gate_mask([1, 0, 2, 1, 5]), [True, False, False, True, False])
    assert SINGLE_PERSON_MIN_FRACTION == 0.8
    assert single_person_frames([1] * 8 + [0, 2]).tolist() == list(range(8))    # 8 / 10: kept
    assert single_person_frames([1] * 7 + [0, 2, 3]) is None                    # 7 / 10: rejected


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
    """Faster R-CNN (a depth-50, 128-pixel random-weight config) on full frames -> person outputs -> gate -> crops of
    the kept frames, against the instance list, the oracle crop, and the 80 % rule on the detector's own boxes."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle.hmr import vitdet_crop
    from vge import synth
    from vge.extract import tokenhmr_front
    from vge.frcnn import FrcnnConfig, FrcnnDetector
    cfg = FrcnnConfig(depth=50, min_size=128, max_size=213, rpn_pre_topk=300, rpn_post_topk=200)
    sd = synth.make_frcnn_state_dict(cfg)
    b = sd["roi_heads.box_predictor.cls_score.bias"]
    b[0] = 6.0                                          # plenty of person instances
    det = FrcnnDetector(sd, cfg, device=DEV, chunk=8)
    frames = synth.make_frames(5, 10, 256, 256)
    fr = torch.from_numpy(frames).to(DEV)
    out = {k: v.cpu().numpy() for k, v in det.detect(fr).items()}
    for f in range(10):   # person outputs = the instance list's class-0 rows
        d = out["dets"][f, :out["n_dets"][f]]
        pers = d[d[:, 5] == 0]
        assert out["n_person"][f] == int((pers[:, 4] > 0.5).sum())
        for j in range(min(2, len(pers))):
            np.testing.assert_array_equal(out["person"][f, j], pers[j, :5])
    assert out["n_person"].max() > 0
    # force a deterministic mix of gate outcomes on the detector's own boxes
    n2 = np.where(np.arange(10) == 9, 0, 1)
    n2[3] = 2                                           # frame 3: two people; frame 9: nobody
    b2 = np.array([[20 + i, 30, 120 + 5 * i, 230] for i in range(10)], np.float32)
    res = tokenhmr_front(det, fr, detections=(b2, n2))
    assert res is not None
    idx, crops = res
    assert idx.tolist() == [0, 1, 2, 4, 5, 6, 7, 8]
    c = crops.cpu().numpy()
    for j, f in enumerate(idx):
        assert np.array_equal(c[j], vitdet_crop(frames[f], b2[f]))
    n3 = n2.copy()
    n3[0] = 0                                           # one more frame fails: 7 / 10 < 80 % -> rejected
    assert tokenhmr_front(det, fr, detections=(b2, n3)) is None
    det.close()
