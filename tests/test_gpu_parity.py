"""GPU parity: libvge.so (through its C ABI) against the golden vectors of the reference and the oracle.

Tolerances (fp32 path; north star: scores within 1e-4 of the reference eval.py):
  feats 1e-4 abs (z-normalised features), stats 1e-6 rel, embeddings 2e-5 abs,
  AC / TC 1e-4 abs (the bar), centroid counts exact.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module")
def vg():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vge import eval as VE
    from vge import ops
    return VE, ops


MODES = ["f32", "f32x3"]


@pytest.fixture(scope="module", params=MODES)
def real_setup(vg, golden_dataset, request):
    VE, ops = vg
    from vge.data import ACTION_CLASSES, NpzVideoDataset, train_test_split
    paths, ckpt = golden_dataset
    real_ds = NpzVideoDataset(paths["real"], filter_classes=ACTION_CLASSES)
    train_ds, _ = train_test_split(real_ds, train_ratio=0.8, seed=1337)
    store = ops.DeviceFrameStore.from_host(VE.load_frame_store(train_ds.items, paths["real_kp"], False), DEV)
    stats = VE.compute_stats_from_npz(train_ds.items, paths["real_kp"], device=DEV, store=store)
    model = VE.load_model(ckpt, device=DEV, compute=request.param)
    return paths, real_ds, train_ds, store, stats, model


def test_stats_match_reference(real_setup, golden_flow):
    _, _, _, _, stats, _ = real_setup
    mean = stats.mean.cpu().numpy()
    std = stats.std.cpu().numpy()
    np.testing.assert_allclose(mean, golden_flow["stats_mean"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(std, golden_flow["stats_std"], rtol=1e-6, atol=1e-7)


def test_featurize_matches_reference(vg, real_setup, golden_flow):
    VE, ops = vg
    from vge.data import create_dataset_from_generated_meshes, sample_all_windows_npz
    paths, _, _, _, stats, _ = real_setup
    ds = create_dataset_from_generated_meshes(paths["generated_meshes"])
    store = ops.DeviceFrameStore.from_host(VE.load_frame_store(ds.items, paths["generated_kps"], True), DEV)
    samples = sample_all_windows_npz(ds)
    idx = {it.path: i for i, it in enumerate(ds.items)}
    win = VE._window_tensor(samples, idx, DEV)
    feats = ops.featurize(store, win, stats.mean, stats.std).cpu().numpy()
    for wi, ref in zip(golden_flow["feat_windows"], golden_flow["feats_sel"]):
        err = np.abs(feats[wi] - ref).max()
        assert err < 1e-4, (wi, err)
    absmean = np.abs(feats).mean(axis=(1, 2))
    np.testing.assert_allclose(absmean, golden_flow["feats_absmean"], rtol=1e-5)


def test_featurize_matches_oracle_all_windows(vg, real_setup):
    """Every generated window (short clips, tail padding, kp shorter than mesh) vs the oracle."""
    VE, ops = vg
    from oracle import featurize as OF
    from oracle.featurize import Stats
    from vge.data import create_dataset_from_generated_meshes, load_clip, sample_all_windows_npz
    paths, _, _, _, stats, _ = real_setup
    ds = create_dataset_from_generated_meshes(paths["generated_meshes"])
    store = ops.DeviceFrameStore.from_host(VE.load_frame_store(ds.items, paths["generated_kps"], True), DEV)
    samples = sample_all_windows_npz(ds)
    idx = {it.path: i for i, it in enumerate(ds.items)}
    feats = ops.featurize(store, VE._window_tensor(samples, idx, DEV), stats.mean, stats.std).cpu().numpy()
    mean, std = stats.mean.cpu().numpy(), stats.std.cpu().numpy()
    for wi, (it, s) in enumerate(samples):
        c = load_clip(it, paths["generated_kps"], True)
        ref = OF.featurize_window(c["pose"], c["global_orient"], c["betas"], c["vit"], c["keypoints"], s, None)
        ref = (ref - mean) / (std + np.float32(1e-6))
        err = np.abs(feats[wi] - ref).max()
        assert err < 1e-4, (wi, it.name, s, err)


def test_encoder_matches_reference(vg, real_setup, golden_flow):
    VE, ops = vg
    from vge.data import create_dataset_from_generated_meshes
    paths, _, _, _, stats, model = real_setup
    ds = create_dataset_from_generated_meshes(paths["generated_meshes"])
    f = VE.extract_window_features(model, ds, paths["generated_kps"], stats, device=DEV, frame_embed=True)
    seq = f["seq_embeds"].cpu().numpy()
    fe = f["frame_embeds"].cpu().numpy()
    assert np.abs(seq - golden_flow["seq_embeds"]).max() < 2e-5
    assert np.abs(fe[:4] - golden_flow["frame_embeds_first4"]).max() < 2e-5


@pytest.mark.parametrize("compute", MODES)
def test_encoder_vs_oracle_random_batch(vg, golden_state_dict, compute):
    """Odd batch (last conv workgroup half empty), random z-scored input, vs the torch-fp32 oracle."""
    VE, ops = vg
    from oracle.encoder import OracleEncoder
    from vge import synth
    torch.manual_seed(0)
    x = torch.randn(37, 32, 2596)
    model = VE.load_model(golden_state_dict, device=DEV, compute=compute)
    seq, fe, tcw = model.encode(x.to(DEV), frame_embed=True, tc=True)
    o = OracleEncoder(golden_state_dict, synth.DIMS_RAW, synth.DIMS_DIFF)
    rs, rf, _ = o.forward(x)
    assert (seq.cpu() - rs).abs().max().item() < 2e-5
    assert (fe.cpu() - rf).abs().max().item() < 2e-5
    f = rf[:, 1:]
    ref_tc = (f[:, 1:] - f[:, :-1]).pow(2).sum(-1).sqrt().mean(-1)
    assert (tcw.cpu() - ref_tc).abs().max().item() < 1e-5
    # the standalone TC kernel on the same frame embeddings
    assert (ops.tc_windows(fe).cpu() - ref_tc).abs().max().item() < 1e-5


def test_centroids_match_reference(vg, real_setup, golden_flow, golden_meta):
    VE, ops = vg
    paths, real_ds, train_ds, store, stats, model = real_setup
    label_dict = {c: i for i, c in enumerate(sorted({it.cls for it in real_ds.items}))}
    assert label_dict == golden_meta["label_dict"]
    cents, ld, counts = VE.build_real_centroids(model, paths["real"], paths["real_kp"], stats, device=DEV,
                                                train_items=train_ds.items, label_dict=label_dict, store=store)
    assert np.array_equal(counts.cpu().numpy(), golden_flow["counts"])
    assert np.abs(cents.cpu().numpy() - golden_flow["centroids"]).max() < 2e-5


@pytest.mark.parametrize("compute", MODES + ["f16"])
def test_video_scores_match_reference(vg, golden_dataset, golden_meta, tmp_path, compute):
    """The whole eval.py flow -> video_scores.json within 1e-4 of the reference (the f16 throughput mode too: its
    fp16 operand rounding stays inside the north-star bar on this set)."""
    VE, ops = vg
    paths, ckpt = golden_dataset
    out = tmp_path / "video_scores.json"
    combined = VE.run_eval(paths["generated_meshes"], paths["real"], ckpt, paths["generated_kps"], paths["real_kp"],
                           out_json=str(out), device=DEV, compute=compute)
    ref = golden_meta["video_scores"]
    assert sorted(combined) == sorted(ref)
    worst = 0.0
    for v, e in ref.items():
        assert set(e) == set(combined[v]), v          # "Testmodel" video: tc only, no ac
        for k in e:
            worst = max(worst, abs(e[k] - combined[v][k]))
    print(f"{compute}: max |score - reference| = {worst:.2e}")
    assert worst < 1e-4, worst
    import json
    assert json.loads(out.read_text()) == combined


def test_cli_with_saved_features(vg, golden_dataset, golden_flow, golden_meta, tmp_path):
    """python -m vge.eval (eval.py's __main__ with arguments): video_scores.json + window_features.pt in the
    reference's format (eval.py:197-204: CPU tensors seq_embeds [Nw,256], frame_embeds [Nw,33,256], names)."""
    VE, ops = vg
    paths, ckpt = golden_dataset
    out, feats = tmp_path / "video_scores.json", tmp_path / "window_features.pt"
    assert VE.main(["--generated-meshes", paths["generated_meshes"], "--real-meshes", paths["real"], "--model", ckpt,
                    "--keypoints", paths["generated_kps"], "--real-keypoints", paths["real_kp"], "--out", str(out),
                    "--save-features", str(feats)]) == 0
    import json
    scores = json.loads(out.read_text())
    ref = golden_meta["video_scores"]
    assert sorted(scores) == sorted(ref)
    assert max(abs(ref[v][k] - scores[v][k]) for v in ref for k in ref[v]) < 1e-4
    f = torch.load(str(feats), weights_only=True)
    assert set(f) == {"seq_embeds", "frame_embeds", "cls_names", "vid_names"}
    assert f["seq_embeds"].device.type == "cpu" and tuple(f["frame_embeds"].shape[1:]) == (33, 256)
    assert np.abs(f["seq_embeds"].numpy() - golden_flow["seq_embeds"]).max() < 2e-5
    assert np.abs(f["frame_embeds"][:4].numpy() - golden_flow["frame_embeds_first4"]).max() < 2e-5
    assert len(f["vid_names"]) == f["seq_embeds"].shape[0]


def test_featurize_edge_cases_vs_oracle(vg):
    """Static / all-invisible / partly invisible keypoints, start past the end, single-frame clip, and an npz shorter
    than its keypoints.npy (the single-person gate keeps 27 of 32 frames: mesh_generator.py:101-117 saves the kept
    frames only, process_video.py every frame; _try_one slices / pads each array on its own)."""
    VE, ops = vg
    from oracle import featurize as OF
    from vge import synth
    from vge.data import pack_frame_store
    rng = np.random.default_rng(5)
    clips = []
    base = synth.make_clip(11, 0, 40)
    for variant in range(5):
        c = synth.make_clip(11, variant, 40 if variant != 4 else 1)
        kp = c.keypoints.copy()
        if variant == 0:
            kp = np.repeat(kp[:1], kp.shape[0], 0)        # static: H = X^T X
        elif variant == 1:
            kp[:] = -1.0                                  # all invisible: H = 0 -> R = I
        elif variant == 2:
            kp[3] = -1.0                                  # one fully invisible frame
        clips.append({"pose": c.pose, "global_orient": c.global_orient, "betas": c.betas, "vit": c.vit,
                      "keypoints": kp})
    c = synth.make_clip(11, 5, 32)
    clips.append({"pose": c.pose[:27], "global_orient": c.global_orient[:27], "betas": c.betas[:27], "vit": c.vit[:27],
                  "keypoints": c.keypoints})
    st = pack_frame_store(clips, [f"c{i}" for i in range(6)], ["X"] * 6)
    store = ops.DeviceFrameStore.from_host(st, DEV)
    wins = [(0, 0), (0, 8), (1, 0), (2, 0), (3, 8), (3, 39), (3, 100), (4, 0), (5, 0)]
    w = torch.tensor(wins, dtype=torch.int32, device=DEV)
    mean = torch.zeros(2596, device=DEV)
    std = torch.full((2596,), 1.0 - 1e-6, device=DEV)
    feats = ops.featurize(store, w, mean, std).cpu().numpy()
    for k, (v, s) in enumerate(wins):
        c = clips[v]
        ref = OF.featurize_window(c["pose"], c["global_orient"], c["betas"], c["vit"], c["keypoints"], s, None)
        ref = ref / (np.float32(1.0 - 1e-6) + np.float32(1e-6))
        err = np.abs(feats[k] - ref).max()
        assert err < 1e-4, (v, s, err)


def test_x3_stem_out_of_fp16_range(vg, golden_state_dict):
    """z-scored columns far outside the fp16 range (train-set std ~ 0): the split path scales stem rows by
    powers of two, so it must still match the torch-fp32 oracle."""
    VE, ops = vg
    from oracle.encoder import OracleEncoder
    from vge import synth
    torch.manual_seed(1)
    x = torch.randn(6, 32, 2596)
    x[:, :, 100:110] *= 3e5          # pose block (raw), beyond 65504
    x[1, 5, 1500] = 2e6               # one diff feature
    x[2] *= 1e-6                      # a whole window of tiny values
    model = VE.load_model(golden_state_dict, device=DEV, compute="f32x3")
    seq, fe, _ = model.encode(x.to(DEV), frame_embed=True, tc=True)
    o = OracleEncoder(golden_state_dict, synth.DIMS_RAW, synth.DIMS_DIFF)
    rs, rf, _ = o.forward(x)
    assert torch.isfinite(seq).all()
    assert (seq.cpu() - rs).abs().max().item() < 1e-4
    assert (fe.cpu() - rf).abs().max().item() < 1e-4


def test_x3_large_weights_and_nonfinite(vg, golden_state_dict):
    """Per-column power-of-two weight scaling: a weight far outside the fp16 range still matches the exact-f32
    path; a non-finite weight cannot be split and is refused loudly (the f32 path takes it)."""
    VE, ops = vg
    from vge.lib import VgeError
    sd = {k: v.copy() for k, v in golden_state_dict.items()}
    k = next(k for k in sd if k.endswith("proj.weight"))
    sd[k][0, 0] = 1e5
    torch.manual_seed(2)
    x = torch.randn(5, 32, 2596, device=DEV)
    s3, f3, _ = VE.load_model(sd, device=DEV, compute="f32x3").encode(x, frame_embed=True)
    s1, f1, _ = VE.load_model(sd, device=DEV, compute="f32").encode(x, frame_embed=True)
    assert (s3 - s1).abs().max().item() < 2e-5
    assert (f3 - f1).abs().max().item() < 2e-5
    sd[k][0, 1] = np.inf
    with pytest.raises(VgeError, match="non-finite"):
        VE.load_model(sd, device=DEV, compute="f32x3")


@pytest.mark.parametrize("n", [37, 256, 293, 600])
def test_x3_quad_and_pair_blocks_vs_f32(vg, golden_state_dict, n):
    """Large batches run the conv chain in 4-window (quad) blocks with 2-window blocks filling the last round
    (37: pairs and a half-empty pair; 256: quads + a round of pairs; 293: quads + one half-empty pair; 600: quads
    only).  Checked against the exact-f32 MFMA path (itself pinned to the oracle above) on the same input."""
    VE, ops = vg
    torch.manual_seed(n)
    x = torch.randn(n, 32, 2596, device=DEV)
    x[:, :, 40:48] *= 1e4   # a few large z-scores: per-row / per-window scaling at work
    s3, f3, t3 = VE.load_model(golden_state_dict, device=DEV, compute="f32x3").encode(x, frame_embed=True, tc=True)
    s1, f1, t1 = VE.load_model(golden_state_dict, device=DEV, compute="f32").encode(x, frame_embed=True, tc=True)
    assert (s3 - s1).abs().max().item() < 2e-5
    assert (f3 - f1).abs().max().item() < 2e-5
    assert (t3 - t1).abs().max().item() < 1e-5


def _encoder_images(enc):
    import ctypes as C
    lib = enc._lib
    lib.vge_debug_encoder_images.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t),
                                             C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
    hb, nh, wb, nf = C.c_void_p(), C.c_size_t(), C.c_void_p(), C.c_size_t()
    assert lib.vge_debug_encoder_images(enc._h, C.byref(hb), C.byref(nh), C.byref(wb), C.byref(nf)) == 0
    h = torch.empty(nh.value, dtype=torch.int16, device=DEV)
    w = torch.empty(nf.value, dtype=torch.int32, device=DEV)
    torch.cuda.synchronize()
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    assert hip.hipMemcpy(h.data_ptr(), hb.value, nh.value * 2, 3) == 0  # hipMemcpyDeviceToDevice
    assert hip.hipMemcpy(w.data_ptr(), wb.value, nf.value * 4, 3) == 0
    torch.cuda.synchronize()
    return h.cpu(), w.cpu()


@pytest.mark.gpu
@pytest.mark.parametrize("big", [False, True])
def test_x3_device_packing_matches_host_packing(vg, golden_state_dict, big, monkeypatch):
    """vge_encoder_create packs the 3xfp16 weight image (hi/lo planes, column exponents, chunk layout) on the
    device; VGE_HOST_PACK=1 runs the host packer.  Both images (fp16 chunks and the f32 image holding the column
    scales) must be identical bit for bit, including a column far outside the fp16 range."""
    VE, ops = vg
    sd = {k: v.copy() for k, v in golden_state_dict.items()}
    if big:
        k = next(k for k in sd if k.endswith("proj.weight"))
        sd[k][3, 7] = 1e5
        k = next(k for k in sd if k.endswith("conv1.weight"))
        sd[k][5, 9, 2] = 3e-9
    dev_enc = VE.load_model(sd, device=DEV, compute="f32x3")
    monkeypatch.setenv("VGE_HOST_PACK", "1")
    host_enc = VE.load_model(sd, device=DEV, compute="f32x3")
    hd, wd = _encoder_images(dev_enc)
    hh, wh = _encoder_images(host_enc)
    assert hd.numel() > 10_000_000 and torch.equal(hd, hh)
    assert torch.equal(wd, wh)


@pytest.mark.parametrize("n,C", [(60_000, 10), (1_000, 70), (5, 3)])
def test_centroid_segmented_reduction_vs_index_add(vg, n, C):
    """build_train_centroids_subset (utils.py:1018-1045) at TAG-Bench-size real sets: the segmented device
    reduction vs torch index_add_ on the host (counts exact, centroids within 2e-5); two launches give the same
    bits; a second accumulate adds onto the first (the ABI accumulates into sums / counts)."""
    VE, ops = vg
    g = torch.Generator().manual_seed(n + C)
    seq = torch.nn.functional.normalize(torch.randn(n, 256, generator=g), dim=-1)
    y = torch.randint(0, C, (n,), generator=g)
    ref_s = torch.zeros(C, 256).index_add_(0, y, seq)
    ref_c = torch.zeros(C).index_add_(0, y, torch.ones(n))
    ref = torch.nn.functional.normalize(ref_s / ref_c.clamp_min(1).unsqueeze(1), dim=-1)
    ds, dy = seq.to(DEV), y.to(torch.int32).to(DEV)
    outs = []
    for _ in range(2):
        s = torch.zeros(C, 256, device=DEV)
        c = torch.zeros(C, device=DEV)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        ops.centroid_accumulate(ds, dy, s, c)
        ev[1].record()
        torch.cuda.synchronize()
        outs.append((s.cpu(), c.cpu(), ev[0].elapsed_time(ev[1])))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    s, c, ms = outs[1]
    assert torch.equal(c, ref_c)
    assert (s - ref_s).abs().max().item() < 1e-3
    cent = ops.centroid_finalize(s.to(DEV), c.to(DEV)).cpu()
    assert (cent - ref).abs().max().item() < 2e-5
    print(f"centroid_accumulate n={n} C={C}: {ms * 1e3:.1f} us")
    s2, c2 = s.to(DEV).clone(), c.to(DEV).clone()
    ops.centroid_accumulate(ds, dy, s2, c2)
    assert torch.equal(c2.cpu(), 2 * ref_c)


def test_cli_explicit_keypoint_layouts(vg, golden_dataset, golden_meta, tmp_path):
    """--kp-layout / --real-kp-layout: the golden keypoint dirs copied under names the reference's sniffing rule
    (utils.py:410-417) would misread; with the layouts stated the scores equal the reference's."""
    import json
    import shutil
    from vge import data
    VE, ops = vg
    paths, ckpt = golden_dataset
    gen_kp, real_kp = tmp_path / "gen_keypoints", tmp_path / "real_keypoints"
    shutil.copytree(paths["generated_kps"], gen_kp)
    shutil.copytree(paths["real_kp"], real_kp)
    out = tmp_path / "video_scores.json"
    try:
        assert VE.main(["--generated-meshes", paths["generated_meshes"], "--real-meshes", paths["real"],
                        "--model", ckpt, "--keypoints", str(gen_kp), "--real-keypoints", str(real_kp),
                        "--kp-layout", "flat", "--real-kp-layout", "per_class", "--out", str(out)]) == 0
    finally:
        data.clear_keypoint_layouts()
    scores = json.loads(out.read_text())
    ref = golden_meta["video_scores"]
    assert sorted(scores) == sorted(ref)
    assert max(abs(ref[v][k] - scores[v][k]) for v in ref for k in ref[v]) < 1e-4


def test_conv_exchange_timeout_raises_device_fault(vg, golden_state_dict):
    """The staggered conv kernel's half-workgroup exchange wait is bounded; a wave that gives up raises the encoder's
    status word, and the library reports VGE_ERR_DEVICE (DeviceFaultError) instead of returning its wrong embeddings
    silently.  A spin bound of 0 forces the give-up on the real kernel; the bound restored and the word cleared, the
    same encoder is correct again."""
    VE, ops = vg
    from vge import lib as L
    so = L.load()
    torch.manual_seed(3)
    x = torch.randn(256, 32, 2596, device=DEV)
    enc = VE.load_model(golden_state_dict, device=DEV, compute="f32x3")
    good, _, _ = enc.encode(x)
    torch.cuda.synchronize()
    enc.status()
    so.vge_debug_set_x3s_spin_limit(0)
    try:
        enc.encode(x)
        torch.cuda.synchronize()
    finally:
        so.vge_debug_set_x3s_spin_limit(-1)
    with pytest.raises(L.DeviceFaultError):
        enc.status()
    with pytest.raises(L.DeviceFaultError):  # later encodes refuse to run until the word is cleared
        enc.encode(x)
    enc.clear_status()
    again, _, _ = enc.encode(x)
    torch.cuda.synchronize()
    enc.status()
    assert torch.equal(good, again)


def test_device_fault_in_the_last_encode_stops_run_eval(vg, golden_dataset, tmp_path):
    """a fault in the last (here: the only) encode of a flow has no later vge_encode to report it; the flow
    checks the status word after its final synchronize, so run_eval raises DeviceFaultError instead of writing scores
    computed from wrong embeddings.  The golden set is one batch (< 1024 windows) per phase."""
    VE, _ = vg
    from vge import lib as L
    so = L.load()
    paths, ckpt = golden_dataset
    out = tmp_path / "scores.json"
    so.vge_debug_set_x3s_spin_limit(0)
    try:
        with pytest.raises(L.DeviceFaultError):
            VE.run_eval(paths["generated_meshes"], paths["real"], ckpt, paths["generated_kps"], paths["real_kp"],
                        out_json=str(out), device=DEV, compute="f32x3")
    finally:
        so.vge_debug_set_x3s_spin_limit(-1)
    assert not out.exists()
