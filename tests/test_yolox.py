"""DWPose's YOLOX person detector (include/vge_dwpose.h vge_yolox_*; vge_yolox.cpp, vge_cnn.hip,
vge_pose_head.hip) against oracle/yolox.py, and the Wholebody composition (detector -> pose model -> rows).

Parity vs the upstream yolox_l.onnx is UNPINNED (not in the reference, no weights offline).  Checked:
  network + decode   every anchor's decoded box / score vs the oracle with the same bf16 storage points: scores
                     within 2e-2 abs, box corners within 2e-2 relative to the box size (+0.5 px)
  NMS + filter       the two persons and min(count, 2) equal EXACTLY the oracle's greedy NMS run on the GPU's own
                     decoded anchors
"""
import numpy as np
import pytest
import torch

DEV = "cuda:0"
gpu = pytest.mark.gpu


def _small():
    from vge.dwpose import YoloxConfig
    return YoloxConfig(in_size=128, width=16, depth=1, head_ch=64)


# ------------------------------------------------------------------------------ CPU
def test_letterbox_focus_layout():
    from oracle.yolox import letterbox_focus
    fr = np.random.default_rng(0).integers(0, 256, (64, 64, 3), dtype=np.uint8)
    x = letterbox_focus(fr, 64)       # r = 1: the frame itself, BGR, Focus space-to-depth
    bgr = fr[..., ::-1].astype(np.float32).transpose(2, 0, 1)
    np.testing.assert_array_equal(x[0:3], bgr[:, ::2, ::2])
    np.testing.assert_array_equal(x[3:6], bgr[:, 1::2, ::2])
    np.testing.assert_array_equal(x[6:9], bgr[:, ::2, 1::2])
    np.testing.assert_array_equal(x[9:12], bgr[:, 1::2, 1::2])
    y = letterbox_focus(fr[:32], 64)  # 32 x 64 -> r = 1, rows 32.. are the 114 padding
    assert (y[:, 16:] == 114).all()


def test_two_person_nms_rules():
    from oracle.yolox import iou_plus1, two_persons
    b = np.array([[0, 0, 100, 100], [5, 5, 105, 105], [200, 0, 260, 90], [0, 0, 10, 10]], np.float32)
    s = np.array([0.9, 0.8, 0.5, 0.95], np.float32)
    kept, n = two_persons(b, s)
    # 3 (0.95) first; 0 (0.9) does not overlap it more than 0.45 -> second
    assert n == 2 and np.array_equal(kept, b[[3, 0]])
    assert iou_plus1(b[0], b[1]) > 0.45
    kept, n = two_persons(b[:3], s[:3])      # 1 is suppressed by 0 -> 2 is the second person
    assert n == 2 and np.array_equal(kept, b[[0, 2]])
    kept, n = two_persons(b[:2], s[:2])
    assert n == 1
    kept, n = two_persons(b, np.full(4, 0.3, np.float32))   # score must be > 0.3
    assert n == 0 and kept.shape == (0, 4)


def test_yolox_config_and_weights_checked_without_gpu_work():
    import ctypes as C
    from vge import dwpose as D
    from vge import lib as L
    from vge import synth
    lib = D._sig(L.load())
    out = C.c_void_p()
    bad = D._ycfg_c(D.YoloxConfig(in_size=100))
    assert lib.vge_yolox_create(C.byref(bad), None, 0, C.byref(out)) == 1
    cfg = _small()
    sd = synth.make_yolox_state_dict(cfg)
    del sd["head.obj_preds.2.bias"]
    keep, arr, n = D._views(sd)
    assert lib.vge_yolox_create(C.byref(D._ycfg_c(cfg)), arr, n, C.byref(out)) == 3
    assert b"head.obj_preds.2.bias" in lib.vge_last_error()


def test_flops_match_published_yolox_l():
    from vge.dwpose import yolox_flops
    assert abs(yolox_flops() / 1e9 - 155.0) < 2.0   # YOLOX-L: 155.6 GFLOPs at 640 (80 classes)


# ------------------------------------------------------------------------------ GPU
@pytest.fixture(scope="module")
def D():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vge import dwpose
    return dwpose


@gpu
@pytest.mark.parametrize("full", [False, True])
def test_detector_vs_oracle(D, full):
    from oracle.yolox import OracleYolox, decode, two_persons
    from vge import synth
    cfg = D.YOLOX_L if full else _small()
    sd = synth.make_yolox_state_dict(cfg)
    frames = synth.make_frames(7, 3, 240, 320)            # letterbox with 114 padding rows
    det = D.YoloxDetector(sd, cfg, device=DEV, chunk=2)    # 2 chunks
    cand = torch.empty((3, det.anchors, 5), device=DEV)
    boxes, npers = det.detect(torch.from_numpy(frames).to(DEV), cand=cand)
    boxes, npers, cand = boxes.cpu().numpy(), npers.cpu().numpy(), cand.cpu().numpy()
    ob, os_ = decode(OracleYolox(sd, cfg, bf16=True).forward(frames), frames.shape[1:3], cfg.in_size)
    serr = float(np.abs(cand[..., 4] - os_).max())
    size = np.maximum(ob[..., 2] - ob[..., 0], ob[..., 3] - ob[..., 1])[..., None]
    berr = np.abs(cand[..., :4] - ob) / (size + 1.0)
    print(f"scores max|d| {serr:.2e}, box corners max rel {float(berr.max()):.2e}")
    assert serr < 2e-2
    assert float(np.quantile(berr, 0.999)) < 2e-2 and float(berr.max()) < 0.1
    for f in range(3):
        kept, n = two_persons(cand[f, :, :4], cand[f, :, 4])
        assert int(npers[f]) == n
        np.testing.assert_array_equal(boxes[f, :n], kept)
        assert (boxes[f, n:] == 0).all()


@gpu
def test_wholebody_composition(D):
    """Detector -> host instance table -> pose model: equals calling the pose model with the detector's boxes."""
    from vge import synth
    from vge.dwpose import RtmposeConfig
    ycfg = _small()
    pcfg = RtmposeConfig(in_h=128, in_w=96, stem_ch=16, stage_ch=(32, 64, 128, 256), stage_blocks=(1, 1, 1, 1))
    det = D.YoloxDetector(synth.make_yolox_state_dict(ycfg), ycfg, device=DEV, chunk=4)
    pose = D.DwposeExtractor(synth.make_rtmpose_state_dict(pcfg), pcfg, device=DEV, max_instances=8)
    frames = torch.from_numpy(synth.make_frames(9, 4, 200, 300)).to(DEV)
    rows = D.Wholebody(det, pose)(frames).cpu().numpy()
    boxes, npers = det.detect(frames)
    want = pose.keypoints(frames, boxes.cpu().numpy(), npers.cpu().numpy()).cpu().numpy()
    np.testing.assert_array_equal(rows, want)
    assert rows.shape == (4, 120) and np.isfinite(rows).all()
