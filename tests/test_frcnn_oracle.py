"""CPU checks of oracle/frcnn.py, the restatement of the reference's gate detector (detectron2 Faster R-CNN X101-FPN,
modifications/mesh_generator.py:69-73, 103-117).  detectron2 is absent offline, so the pieces are pinned where an
independent answer exists: the ResizeShortestEdge resample against Pillow itself (the library DefaultPredictor calls),
NMS / batched NMS / ROIAlign / box decoding against hand-computed known answers and direct float64 evaluations of
their definitions.  The network's parity vs detectron2's trained weights stays unpinned."""
import math

import numpy as np
import pytest
import torch

from oracle import frcnn as OF


@pytest.mark.parametrize("h,w,nh,nw", [(256, 256, 800, 800), (100, 37, 800, 296), (480, 640, 800, 1067),
                                       (1000, 900, 800, 720), (31, 57, 45, 83), (64, 64, 64, 64)])
def test_resize_is_pillow_bilinear_bit_exact(h, w, nh, nw):
    from PIL import Image
    img = np.random.default_rng(h * 1000 + w).integers(0, 256, (h, w, 3), dtype=np.uint8)
    want = np.asarray(Image.fromarray(img).resize((nw, nh), Image.BILINEAR))
    np.testing.assert_array_equal(OF.resize_pil(img, nh, nw), want)


def test_resize_shortest_edge_shapes():
    assert OF.output_shape(256, 256, 800, 1333) == (800, 800)
    assert OF.output_shape(480, 640, 800, 1333) == (800, 1067)
    assert OF.output_shape(100, 1000, 800, 1333) == (133, 1333)   # long side capped
    assert OF.output_shape(640, 480, 800, 1333) == (1067, 800)


def test_preprocess_normalises_bgr_and_pads_to_32():
    class Cfg:
        min_size, max_size = 100, 1000
    fr = np.zeros((50, 70, 3), np.uint8)
    fr[..., 0] = 255  # pure red
    x, (nh, nw) = OF.preprocess(fr, Cfg)
    assert (nh, nw) == (100, 140) and x.shape == (3, 128, 160)
    np.testing.assert_allclose(x[:, :nh, :nw].reshape(3, -1).mean(1),
                               [(0 - 103.53) / 57.375, (0 - 116.28) / 57.12, (255 - 123.675) / 58.395], rtol=1e-6)
    assert not x[:, nh:, :].any() and not x[:, :, nw:].any()


def test_cell_anchors_are_detectron2s():
    a = OF.cell_anchors(32, (0.5, 1.0, 2.0))
    np.testing.assert_allclose(a[1], [-16, -16, 16, 16])
    w = math.sqrt(1024 / 0.5)
    np.testing.assert_allclose(a[0], np.float32([-w / 2, -0.5 * w / 2, w / 2, 0.5 * w / 2]))
    g = OF.grid_anchors(2, 3, 8, 32, (0.5, 1.0, 2.0))
    assert g.shape == (18, 4)
    np.testing.assert_allclose(g[3 * 4 + 1].numpy(), [8 * 1 - 16, 8 * 1 - 16, 8 + 16, 8 + 16])  # (y 1, x 1, ratio 1)


def test_apply_deltas_known_answers():
    boxes = torch.tensor([[10., 20., 30., 60.]])
    z = OF.apply_deltas(torch.zeros(1, 8), boxes, (10., 10., 5., 5.))
    np.testing.assert_allclose(z.numpy().reshape(2, 4), [[10, 20, 30, 60]] * 2)
    d = torch.tensor([[2.0, -4.0, 5 * math.log(2.0), 0.0]])   # dx 0.2 w, dy -0.4 h, w x 2
    out = OF.apply_deltas(d, boxes, (10., 10., 5., 5.))[0].numpy()
    cx, cy = 20 + 0.2 * 20, 40 - 0.4 * 40
    np.testing.assert_allclose(out, [cx - 20, cy - 20, cx + 20, cy + 20], rtol=1e-6)
    big = OF.apply_deltas(torch.tensor([[0., 0., 100., 100.]]), boxes, (1., 1., 1., 1.))[0].numpy()
    np.testing.assert_allclose(big[2] - big[0], 20 * 1000 / 16, rtol=1e-5)   # scale clamp log(1000 / 16)


def test_nms_known_answers():
    b = torch.tensor([[0., 0., 10., 10.], [1., 1., 11., 11.], [20., 20., 30., 30.], [0., 0., 10., 10.5]])
    s = torch.tensor([0.9, 0.8, 0.7, 0.95])
    # IoU(3, 0) = 100 / 105 > 0.5 -> 0 suppressed; IoU(3, 1) = 81 / 124 > 0.5 -> 1 suppressed
    assert OF.nms(b, s, 0.5).tolist() == [3, 2]
    assert OF.nms(b, s, 0.96).tolist() == [3, 0, 1, 2]
    # ties: the lower index first
    assert OF.nms(torch.tensor([[0., 0., 1., 1.], [5., 5., 6., 6.]]), torch.tensor([0.5, 0.5]), 0.5).tolist() == [0, 1]
    # batched: class-aware (the overlapping pair survives when the classes differ), output by score
    assert OF.batched_nms(b, s, torch.tensor([0, 1, 0, 0]), 0.5).tolist() == [3, 1, 2]


def _roi_align_f64(feat, box, scale, pooled=7):
    """ROIAlignV2 (aligned, adaptive grid) straight from its definition in float64."""
    C, H, W = feat.shape
    x1, y1, x2, y2 = (float(v) * scale - 0.5 for v in box)
    rw, rh = x2 - x1, y2 - y1
    gh, gw = math.ceil(rh / pooled), math.ceil(rw / pooled)
    out = np.zeros((C, pooled, pooled))
    for ph in range(pooled):
        for pw in range(pooled):
            acc = np.zeros(C)
            for iy in range(gh):
                y = y1 + ph * rh / pooled + (iy + 0.5) * rh / pooled / gh
                for ix in range(gw):
                    x = x1 + pw * rw / pooled + (ix + 0.5) * rw / pooled / gw
                    if y < -1 or y > H or x < -1 or x > W:
                        continue
                    y, x = max(y, 0.0), max(x, 0.0)
                    yl, xl = min(int(y), H - 1), min(int(x), W - 1)
                    yh, xh = min(yl + 1, H - 1), min(xl + 1, W - 1)
                    ly = y - yl if yl < H - 1 else 0.0
                    lx = x - xl if xl < W - 1 else 0.0
                    acc += ((1 - ly) * (1 - lx) * feat[:, yl, xl] + (1 - ly) * lx * feat[:, yl, xh]
                            + ly * (1 - lx) * feat[:, yh, xl] + ly * lx * feat[:, yh, xh])
            out[:, ph, pw] = acc / max(gh * gw, 1)
    return out


def test_roi_align_matches_its_definition():
    rng = np.random.default_rng(3)
    feat = rng.standard_normal((4, 13, 17)).astype(np.float32)
    boxes = torch.tensor([[3.0, 5.0, 40.0, 30.0], [0.0, 0.0, 68.0, 52.0], [20.5, 11.25, 22.0, 60.0],
                          [-8.0, 40.0, 80.0, 70.0]])
    got = OF.roi_align(torch.from_numpy(feat), boxes, 0.25).numpy()
    for r in range(boxes.shape[0]):
        np.testing.assert_allclose(got[r], _roi_align_f64(feat.astype(np.float64), boxes[r].tolist(), 0.25),
                                   rtol=2e-5, atol=2e-5)
    const = OF.roi_align(torch.full((2, 8, 8), 3.5), torch.tensor([[4.0, 4.0, 20.0, 28.0]]), 0.25)
    np.testing.assert_allclose(const.numpy(), 3.5, rtol=1e-6)


def test_level_assignment():
    # floor(4 + log2(sqrt(area) / 224 + 1e-8)) clamped to [2, 5], minus 2
    b = torch.tensor([[0., 0., 224., 224.], [0., 0., 113., 113.], [0., 0., 111., 111.], [0., 0., 10., 10.],
                      [0., 0., 1000., 1000.], [0., 0., 448., 448.]])
    assert OF.assign_levels(b).tolist() == [2, 1, 0, 0, 3, 3]


def test_oracle_detector_runs_end_to_end_small():
    """A depth-50 / 128-pixel instance of the restated predictor: sorted scores above the threshold, classes in range,
    boxes inside the frame, at most det_per_img instances, the gate count."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "video-gen-evals_amd"))
    from vge import synth
    from vge.frcnn import FrcnnConfig
    cfg = FrcnnConfig(depth=50, min_size=128, max_size=213, rpn_pre_topk=300, rpn_post_topk=200)
    o = OF.OracleFrcnn(synth.make_frcnn_state_dict(cfg), cfg, bf16=True)
    fr = synth.make_frame_pool(11, 2, h=96, w=80)
    res = o.detect(fr)
    for r in res:
        s = r["scores"].numpy()
        assert 0 < len(s) <= cfg.det_per_img and (s > cfg.score_thresh).all() and (np.diff(s) <= 0).all()
        assert ((r["classes"] >= 0) & (r["classes"] < cfg.num_classes)).all()
        b = r["boxes"].numpy()
        assert (b[:, 0] >= 0).all() and (b[:, 2] <= 80).all() and (b[:, 3] <= 96).all()
        assert (b[:, 2] > b[:, 0]).all() and (b[:, 3] > b[:, 1]).all()
        assert OF.gate_persons(r) == int(((r["classes"] == 0) & (r["scores"] > 0.5)).sum())


def test_detector_refuses_a_score_threshold_its_candidate_slots_cannot_hold():
    """det_post_kernel keeps 4 candidate classes per proposal, exact only for score_thresh >= 0.2 (five classes above
    0.2 would sum past 1): vge_frcnn_create refuses a lower threshold (detectron2's own default, 0.05, included) with
    VGE_ERR_ARG before touching weights or the GPU; the reference's 0.25 passes the check."""
    import ctypes as C
    import dataclasses
    from vge import lib as L
    from vge.frcnn import FRCNN_X101, _cfg_c, _sig
    so = _sig(L.load())
    for thr in (0.05, 0.19, 1.5):
        h = C.c_void_p()
        cc = _cfg_c(dataclasses.replace(FRCNN_X101, score_thresh=thr))
        assert so.vge_frcnn_create(C.byref(cc), None, 0, C.byref(h)) == 1
        assert b"score_thresh" in so.vge_last_error()
    h = C.c_void_p()
    cc = _cfg_c(FRCNN_X101)
    rc = so.vge_frcnn_create(C.byref(cc), None, 0, C.byref(h))   # no weights: fails on the first missing tensor
    assert rc != 0 and b"score_thresh" not in so.vge_last_error()
