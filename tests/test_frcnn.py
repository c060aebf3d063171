"""GPU parity of TokenHMR's gate detector (detectron2 Faster R-CNN X101-32x8d-FPN, modifications/mesh_generator.py:69-73,
103-117) through the C ABI (include/vge_frcnn.h) against oracle/frcnn.py, at full width and the reference's 800-pixel
input on four 256 x 256 frames (two chunks of the workspace).

Every stage is checked on the GPU's own input to that stage, so a tolerance covers one stage's arithmetic:
  resize        the PIL bilinear resample, byte for byte
  backbone+FPN  P2..P6 vs the oracle run from the frames (bf16 storage points, 101 layers: relative L2 < 3e-2)
  RPN head      logits / deltas from the GPU's P levels (one bf16 conv + f32 1x1)
  proposals     top-k / decode / clip / batched NMS / merge from the GPU's logits: identical order and scores
  ROIAlign      from the GPU's P levels and proposals: torchvision's float order, identical but for rare 1-ulp bf16
  box head      fc1 / fc2 / predictor from the GPU's box features
  inference     softmax / per-class decode / NMS / top 100 / postprocess from the GPU's head: identical instances
  gate          the person count of mesh_generator.py:106-108, and the whole predictor end to end vs the oracle
Parity vs detectron2's trained model is UNPINNED (code and weights absent offline; random weights of the reference's
shapes, vge.synth.make_frcnn_state_dict).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
NF = 4


@pytest.fixture(scope="module")
def run():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle.frcnn import OracleFrcnn
    from vge import synth
    from vge.frcnn import FRCNN_X101, FrcnnDetector
    cfg = FRCNN_X101
    sd = synth.make_frcnn_state_dict(cfg)
    det = FrcnnDetector(sd, cfg, device=DEV, chunk=3)          # 4 frames = two chunks (tap / output offsets)
    frames = synth.make_frame_pool(9100, NF)
    fr = torch.from_numpy(frames).to(DEV)
    taps = det.make_taps(NF, 256, 256)
    out = det.detect(fr, taps=taps)
    torch.cuda.synchronize()
    host = lambda v: [x.cpu() for x in v] if isinstance(v, list) else v.cpu()  # noqa: E731
    r = dict(cfg=cfg, sd=sd, frames=frames, out={k: host(v) for k, v in out.items()},
             taps={k: host(v) for k, v in taps.items()}, shapes=det.shapes(256, 256),
             oracle=OracleFrcnn(sd, cfg, bf16=True))
    det.close()
    return r


@pytest.fixture(scope="module")
def oracle_fwd(run):
    """The oracle predictor from the frames themselves, on the first two frames."""
    torch.set_num_threads(16)
    res, aux = run["oracle"].detect(run["frames"][:2], taps=True)
    return res, aux


def _nchw(t):  # bf16 [F, h, w, C] -> float [F, C, h, w]
    return t.float().permute(0, 3, 1, 2).contiguous()


def test_resize_is_pil_bilinear(run):
    from oracle.frcnn import resize_pil
    nh, nw = run["shapes"]["resized"]
    for f in range(NF):
        np.testing.assert_array_equal(run["taps"]["resized"][f].numpy(), resize_pil(run["frames"][f], nh, nw))


def test_backbone_fpn_vs_oracle(run, oracle_fwd):
    _, aux = oracle_fwd
    for l in range(5):
        g, o = _nchw(run["taps"]["fpn"][l][:2]), aux["P"][l]
        rel = float((g - o).norm() / o.norm())
        mx = float((g - o).abs().max() / o.abs().max())
        print(f"P{l + 2}: rel L2 {rel:.2e}, max |d| / max |ref| {mx:.2e}")
        assert rel < 3e-2 and mx < 0.15, (l, rel, mx)


def test_rpn_head_vs_oracle(run):
    o = run["oracle"]
    for l in range(5):
        P = _nchw(run["taps"]["fpn"][l][:2])
        lo, de = o.rpn_head(P)
        g = run["taps"]["rpn"][l][:2]
        h, w = g.shape[1:3]
        gl = g[..., :3].reshape(2, -1)
        gd = g[..., 3:15].reshape(2, h * w * 3, 4)
        el, ed = float((gl - lo).abs().max()), float((gd - de).abs().max())
        print(f"RPN P{l + 2}: logits max|d| {el:.2e} (max {float(lo.abs().max()):.2f}), deltas {ed:.2e}")
        assert el < 3e-2 * max(1.0, float(lo.abs().max())) and ed < 3e-2 * max(0.1, float(de.abs().max()))


def _gpu_head_inputs(run, f):
    t = run["taps"]
    logits = [t["rpn"][l][f, ..., :3].reshape(-1) for l in range(5)]
    deltas = [t["rpn"][l][f, ..., 3:15].reshape(-1, 4) for l in range(5)]
    return logits, deltas


def test_proposals_vs_oracle_on_gpu_logits(run):
    o, t = run["oracle"], run["taps"]
    shapes = [tuple(s) for s in run["shapes"]["levels"]]
    size = tuple(run["shapes"]["resized"])
    for f in range(NF):
        lo, de = _gpu_head_inputs(run, f)
        pb, ps = o.proposals(lo, de, size, shapes)
        n = int(t["n_proposals"][f])
        gp = t["proposals"][f, :n]
        assert n == pb.shape[0], (f, n, pb.shape[0])
        assert torch.equal(gp[:, 4], ps), f"frame {f}: proposal order / scores differ"
        err = float((gp[:, :4] - pb).abs().max())
        print(f"frame {f}: {n} proposals, max |box d| {err:.2e}")
        assert err < 2e-3


def test_box_features_vs_oracle_on_gpu_levels(run):
    o, t = run["oracle"], run["taps"]
    for f in range(2):
        n = int(t["n_proposals"][f])
        pf = [_nchw(t["fpn"][l][f:f + 1])[0] for l in range(4)]
        ref = o.box_features(pf, t["proposals"][f, :n, :4])                    # [n, 256, 7, 7] (bf16 values)
        got = t["box_features"][f, :n].float().view(n, 7, 7, 256).permute(0, 3, 1, 2)
        d = (got - ref).abs()
        same = float((d == 0).float().mean())
        ulp = float((d / ref.abs().clamp_min(1e-30)).max())
        print(f"frame {f}: ROIAlign bins identical {same:.6f}, max rel diff {ulp:.2e}")
        assert same > 0.999 and float((d - ref.abs() * 2 ** -7).max()) <= 1e-6


def test_roi_align_separable_matches_sample_order(run):
    """The default ROIAlign (separable per-bin cell weights, roi_align_sep_kernel) against torchvision's sample order
    (roi_align_kernel, vge_debug_set_roi_direct) on the same levels and proposals: the same sums reassociated, so
    bins identical but for rare 1-ulp bf16 differences.  The separable kernel's sample-loop branch (taken for bins
    wider than its LDS tables, forced here for every ROI) is roi_align_kernel's arithmetic: identical."""
    import ctypes as C
    from vge import synth
    from vge.frcnn import FrcnnDetector
    frames = torch.from_numpy(synth.make_frame_pool(9100, NF)).to(DEV)
    lib = L_load()
    lib.vge_debug_set_roi_direct.argtypes = [C.c_int]
    got = {}
    det = FrcnnDetector(run["sd"], run["cfg"], device=DEV, chunk=NF)
    try:
        for direct in (0, 1, 2):  # 2: the separable kernel's own sample loop (its branch for very wide bins)
            lib.vge_debug_set_roi_direct(direct)
            taps = det.make_taps(NF, 256, 256)
            det.detect(frames, taps=taps)
            torch.cuda.synchronize()
            got[direct] = (taps["box_features"].cpu(), taps["n_proposals"].cpu())
    finally:
        lib.vge_debug_set_roi_direct(0)
        det.close()
    assert torch.equal(got[0][1], got[1][1])
    assert torch.equal(got[2][0], got[1][0]), "the separable kernel's sample loop differs from roi_align_kernel"
    for f in range(NF):
        n = int(got[0][1][f])
        a, b = got[0][0][f, :n].float(), got[1][0][f, :n].float()
        d = (a - b).abs()
        same = float((d == 0).float().mean())
        print(f"frame {f}: {n} ROIs, bins identical {same:.6f}")
        assert n > 0 and same > 0.999 and float((d - b.abs() * 2 ** -7).max()) <= 1e-6


def test_stem_pool_fused_matches_split(run):
    """The fused stem conv + ReLU + max pool (frcnn_stem_pool_kernel, default) against the stem conv kernel followed by
    the max-pool kernel (vge_debug_set_stem_split): the same MFMA K order and bf16 rounding point, so P2..P6 agree to
    the conv kernel's own summation differences and the gate's person counts are the same."""
    import ctypes as C
    from vge import synth
    from vge.frcnn import FrcnnDetector
    frames = torch.from_numpy(synth.make_frame_pool(9100, NF)).to(DEV)
    lib = L_load()
    lib.vge_debug_set_stem_split.argtypes = [C.c_int]
    got = {}
    det = FrcnnDetector(run["sd"], run["cfg"], device=DEV, chunk=NF)
    try:
        for split in (0, 1):
            lib.vge_debug_set_stem_split(split)
            taps = det.make_taps(NF, 256, 256)
            o = det.detect(frames, taps=taps)
            torch.cuda.synchronize()
            got[split] = ([p.float().cpu() for p in taps["fpn"]], o["n_person"].cpu())
    finally:
        lib.vge_debug_set_stem_split(0)
        det.close()
    for l, (a, b) in enumerate(zip(got[0][0], got[1][0])):
        rel = float((a - b).norm() / b.norm())
        print(f"P{l + 2}: fused vs split rel L2 {rel:.2e}, identical {float((a == b).float().mean()):.4f}")
        assert rel < 1e-2, (l, rel)
    assert torch.equal(got[0][1], got[1][1])


def test_box_head_vs_oracle_on_gpu_features(run):
    o, t, K = run["oracle"], run["taps"], run["cfg"].num_classes
    for f in range(2):
        n = int(t["n_proposals"][f])
        cl, de = o.box_head(t["box_features"][f, :n].float().view(n, 7, 7, 256).permute(0, 3, 1, 2))
        g = t["head"][f, :n]
        ec, ed = float((g[:, :K + 1] - cl).abs().max()), float((g[:, K + 1:5 * K + 1] - de).abs().max())
        print(f"frame {f}: cls logits max|d| {ec:.2e} (max {float(cl.abs().max()):.2f}), deltas {ed:.2e}")
        assert ec < 3e-2 * max(1.0, float(cl.abs().max())) and ed < 3e-2 * max(0.1, float(de.abs().max()))


def test_inference_and_postprocess_vs_oracle_on_gpu_head(run):
    from oracle.frcnn import OracleFrcnn, gate_persons
    o, t, out, K = run["oracle"], run["taps"], run["out"], run["cfg"].num_classes
    size = tuple(run["shapes"]["resized"])
    checked = 0
    for f in range(NF):
        n = int(t["n_proposals"][f])
        cl, de = t["head"][f, :n, :K + 1], t["head"][f, :n, K + 1:5 * K + 1]
        e = torch.exp(cl - cl.max(1, keepdim=True).values)
        p = e / e.sum(1, keepdim=True)
        if bool(((p[:, :K] - run["cfg"].score_thresh).abs() < 1e-5).any()):
            print(f"frame {f}: a class probability within 1e-5 of the threshold: skipped")
            continue
        b, s, k = o.inference(cl, de, t["proposals"][f, :n, :4], size)
        m = int(t["n_pre_dets"][f])
        g = t["pre_dets"][f, :m]
        assert m == b.shape[0], (f, m, b.shape[0])
        assert torch.equal(g[:, 5].long(), k), f"frame {f}: classes / order differ"
        np.testing.assert_allclose(g[:, 4].numpy(), s.numpy(), rtol=2e-6, atol=1e-7)
        np.testing.assert_allclose(g[:, :4].numpy(), b.numpy(), rtol=1e-5, atol=2e-3)
        fb, fs, fk = OracleFrcnn.postprocess(b, s, k, size, 256, 256)
        nd = int(out["n_dets"][f])
        assert nd == fb.shape[0]
        np.testing.assert_allclose(out["dets"][f, :nd, :4].numpy(), fb.numpy(), rtol=1e-5, atol=1e-3)
        assert torch.equal(out["dets"][f, :nd, 5].long(), fk)
        assert int(out["n_person"][f]) == gate_persons({"classes": fk, "scores": fs})
        pers = fk == 0
        for j in range(min(2, int(pers.sum()))):
            np.testing.assert_allclose(out["person"][f, j, :4].numpy(), fb[pers][j].numpy(), rtol=1e-5, atol=1e-3)
        checked += 1
        print(f"frame {f}: {m} instances, {int(out['n_person'][f])} persons > 0.5, classes {k[:8].tolist()}")
    assert checked >= 2


def test_predictor_end_to_end_vs_oracle(run, oracle_fwd):
    """The whole predictor from the frames: the oracle's instances are found among the GPU's (same class, IoU > 0.9,
    score within 0.05) and the gate's person count agrees unless an oracle person score is within 0.05 of 0.5."""
    res, _ = oracle_fwd
    out = run["out"]
    from oracle.frcnn import gate_persons
    for f, r in enumerate(res):
        nd = int(out["n_dets"][f])
        g = out["dets"][f, :nd]
        top = min(20, len(r["scores"]))
        hit = 0
        for j in range(top):
            bo = r["boxes"][j]
            same = g[g[:, 5].long() == int(r["classes"][j])]
            if same.shape[0] == 0:
                continue
            x1 = torch.maximum(same[:, 0], bo[0]); y1 = torch.maximum(same[:, 1], bo[1])
            x2 = torch.minimum(same[:, 2], bo[2]); y2 = torch.minimum(same[:, 3], bo[3])
            inter = (x2 - x1).clamp_min(0) * (y2 - y1).clamp_min(0)
            iou = inter / ((same[:, 2] - same[:, 0]) * (same[:, 3] - same[:, 1]) + (bo[2] - bo[0]) * (bo[3] - bo[1]) - inter)
            ok = (iou > 0.9) & ((same[:, 4] - r["scores"][j]).abs() < 0.05)
            hit += int(bool(ok.any()))
        print(f"frame {f}: {hit}/{top} oracle instances matched; persons gpu {int(out['n_person'][f])} "
              f"oracle {gate_persons(r)}")
        assert hit >= 0.8 * top
        ps = r["scores"][r["classes"] == 0]
        if not bool(((ps - 0.5).abs() < 0.05).any()):
            assert int(out["n_person"][f]) == gate_persons(r)


@pytest.mark.parametrize("gw,stride,C,H,W", [(8, 1, 256, 20, 37), (16, 2, 512, 21, 18), (32, 1, 1024, 13, 11),
                                             (64, 1, 2048, 9, 10), (32, 2, 1024, 14, 13), (64, 2, 2048, 7, 6),
                                             (8, 2, 256, 15, 16), (16, 1, 512, 10, 33),
                                             (32, 1, 1024, 50, 50), (16, 1, 512, 100, 100), (8, 1, 256, 200, 200),
                                             (32, 2, 1024, 100, 100), (16, 2, 512, 200, 200), (32, 1, 1024, 51, 47)])
def test_grouped_conv_kernel_vs_torch(gw, stride, C, H, W):
    """The bottlenecks' grouped 3x3 conv (vge_gconv.hip: + folded bias, ReLU) alone vs torch conv2d(groups = C / gw)
    in f32 on the same bf16 operands: every group width of X101-32x8d (8 .. 64 channels per group), both strides,
    ragged tiles (group widths 8 / 16 run two taps per 16x16x32 MFMA, the ninth against zero weights; 32 / 64 one or
    two MFMAs per tap).  The kernel rounds its f32 sums to bf16 once.  The output tile is picked per shape
    (gc_pick_tile): the detector's 200 / 100 / 50-wide maps at both strides take tiles whose 16-pixel groups run across
    rows (5 x 25, 6 x 10), the small shapes whole-image tiles, 51 x 47 a partial last group."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ctypes as C_
    import torch.nn.functional as F
    from vge import lib as L
    so = L.load()
    g = torch.Generator().manual_seed(gw * 7 + stride)
    x = torch.randn((2, H, W, C), generator=g).to(torch.bfloat16)
    w = (torch.randn((C, gw, 3, 3), generator=g) / (3.0 * gw ** 0.5)).float()
    b = (0.1 * torch.randn(C, generator=g)).float()
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    xd = x.to(DEV)
    out = torch.full((2, Ho, Wo, C), float("nan"), dtype=torch.bfloat16, device=DEV)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream().cuda_stream
    rc = so.vge_debug_gconv3(C_.c_void_p(xd.data_ptr()), 2, H, W, C, gw, stride, C_.c_void_p(w.data_ptr()),
                             C_.c_void_p(b.data_ptr()), C_.c_void_p(out.data_ptr()), C_.c_void_p(st))
    assert rc == 0, L.load().vge_last_error()
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.to(torch.bfloat16).float(), b, stride=stride, padding=1,
                   groups=C // gw).relu().permute(0, 2, 3, 1)
    got = out.float().cpu()
    assert torch.isfinite(got).all()
    err = (got - ref).abs()
    bound = 2.0 ** -7 * ref.abs() + 1e-4          # one bf16 rounding of the output (+ f32 summation order)
    print(f"gw {gw} stride {stride}: max |d| {err.max():.2e}, max |ref| {ref.abs().max():.2e}")
    assert bool((err <= bound).all()), float((err - bound).max())


def test_chunk_cap_and_128_frame_chunk_matches_64(run):
    """Activations are addressed through 64-bit offsets (the 1x1 convs' GEMM epilogue included), so a chunk is bounded
    only by int32 row / thread counts: 838 frames at 800 px (vge_frcnn_reserve refuses one more before allocating).
    A 128-frame chunk -- T1 of res3.0's conv1 then holds 2.6e9 elements, past the old 2 GiB cap of 104 frames -- gives
    the same detections, bit for bit, as the same frames in 64-frame chunks (every kernel is per frame or per output
    element with a fixed K order, and the tuner's conv variants are bit-identical).  Run with the library path off:
    hipBLASLt's stream-K algorithms split a GEMM's K loop by its tile count, so the library's 1x1 convs are not
    bit-stable across M (test_chunk_128_with_library_gemms_matches_64 bounds them instead)."""
    import ctypes as C
    from vge import synth
    from vge.frcnn import FrcnnDetector
    frames = torch.from_numpy(synth.make_frame_pool(9300, 128)).to(DEV)
    outs = {}
    lib = L_load()
    lib.vge_debug_set_gemm_lib.argtypes = [C.c_int]
    lib.vge_debug_set_gemm_lib(0)
    for chunk in (128, 64):
        det = FrcnnDetector(run["sd"], run["cfg"], device=DEV, chunk=chunk)
        try:
            if chunk == 128:
                cap = det.max_chunk(256, 256)
                assert cap == 838, cap
                assert det.lib.vge_frcnn_reserve(det.h, cap + 1, 256, 256) == 1      # VGE_ERR_ARG, nothing allocated
            assert det.chunk == chunk
            o = det.detect(frames)
            torch.cuda.synchronize()
            outs[chunk] = {k: v.cpu() for k, v in o.items()}
        finally:
            det.close()
            if chunk == 64:
                lib.vge_debug_set_gemm_lib(1)
        torch.cuda.empty_cache()
    for k in outs[64]:
        assert torch.equal(outs[128][k], outs[64][k]), k
    print(f"128-frame chunk == 2 x 64: {int(outs[64]['n_dets'].sum())} instances, "
          f"{int((outs[64]['n_person'] == 1).sum())} single-person frames")


def L_load():
    from vge import lib as L
    return L.load()


def test_chunk_128_with_library_gemms_matches_64(run):
    """The default path (1x1 convs on hipBLASLt): a 128-frame chunk's FPN maps agree with 64-frame chunks' to the
    library GEMMs' f32 summation-order differences carried through the network (bf16 storage), and the gate's person
    counts agree on every frame whose best person score is not within 0.05 of the gate threshold."""
    from vge import synth
    from vge.frcnn import FrcnnDetector
    frames = torch.from_numpy(synth.make_frame_pool(9300, 128)).to(DEV)
    outs = {}
    for chunk in (128, 64):
        det = FrcnnDetector(run["sd"], run["cfg"], device=DEV, chunk=chunk)
        try:
            taps = det.make_taps(128, 256, 256)
            o = det.detect(frames, taps=taps)
            torch.cuda.synchronize()
            outs[chunk] = ({k: v.cpu() for k, v in o.items()}, [t.float().cpu() for t in taps["fpn"]])
        finally:
            det.close()
        torch.cuda.empty_cache()
    for lv, (a, b) in enumerate(zip(outs[128][1], outs[64][1])):
        rel = float((a - b).abs().max()) / max(float(b.abs().max()), 1e-30)
        print(f"P{lv + 2}: max |d| / max |P| = {rel:.2e}")
        assert rel < 5e-2, (lv, rel)
    d128, d64 = outs[128][0], outs[64][0]
    same = (d128["n_person"] == d64["n_person"])
    assert float(same.float().mean()) >= 0.95, float(same.float().mean())
