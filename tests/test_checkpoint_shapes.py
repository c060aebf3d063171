"""Checkpoints of another shape: load_model builds HumanActionScorer from the checkpoint's own d_model / time_layers /
time_heads (eval.py:136-152), so a d_model 64, 2-layer, 4-head checkpoint must score like the reference.

  CPU  the oracle (oracle/encoder.py at that shape) against tests/golden/golden_flow_small.npz +
       golden_scores_small.json (the reference itself, tests/golden/make_golden.py small); the host-side shape
       handling of vge.eval.load_model
  GPU  libvge's generic exact-f32 path (vge_encoder_gen.hip): embeddings, centroids and video_scores.json within
       1e-4 of the reference; the tiled modes refuse the shape (VGE_ERR_UNSUPPORTED) rather than compute it wrong
"""
import json

import numpy as np
import pytest
import torch

gpu = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def small_state_dict():
    from tests.golden.dataset_spec import golden_state_dict
    return golden_state_dict("small")


@pytest.fixture(scope="module")
def oracle_run_small(golden_dataset_small, small_state_dict, golden_meta_small):
    from oracle import evalflow
    from tests.golden.dataset_spec import SMALL_HP
    from vge import synth
    paths, _ = golden_dataset_small
    return evalflow.run_eval(paths["real"], paths["real_kp"], paths["generated_meshes"], paths["generated_kps"],
                             small_state_dict, synth.DIMS_RAW, synth.DIMS_DIFF, hp=SMALL_HP)


def test_golden_small_shape(golden_flow_small, golden_meta_small):
    assert golden_meta_small["hp"] == {"d_model": 64, "time_layers": 2, "time_heads": 4}
    assert golden_flow_small["seq_embeds"].shape[1] == 64
    assert golden_flow_small["frame_embeds_first4"].shape[1:] == (33, 64)
    assert golden_flow_small["centroids"].shape[1] == 64


def test_oracle_small_embeddings(oracle_run_small, golden_flow_small, golden_meta_small):
    _, ex = oracle_run_small
    assert ex["label_dict"] == golden_meta_small["label_dict"]
    assert np.array_equal(ex["counts"].numpy(), golden_flow_small["counts"])
    assert np.abs(ex["centroids"].numpy() - golden_flow_small["centroids"]).max() < 1e-5
    assert np.abs(ex["seq"].numpy() - golden_flow_small["seq_embeds"]).max() < 1e-5
    assert np.abs(ex["frame_embeds"][:4].numpy() - golden_flow_small["frame_embeds_first4"]).max() < 1e-5


def test_oracle_small_scores(oracle_run_small, golden_meta_small):
    combined, _ = oracle_run_small
    ref = golden_meta_small["video_scores"]
    assert sorted(combined) == sorted(ref)
    assert max(abs(ref[v][k] - combined[v][k]) for v in ref for k in ref[v]) < 1e-5


def test_load_model_reads_the_checkpoint_shape(golden_dataset_small, monkeypatch, tmp_path):
    """load_model passes the checkpoint's hyper-parameters and picks the exact-f32 path for a non-(256, 8) shape
    (no GPU: the Encoder constructor is intercepted)."""
    from vge import eval as VE
    from vge import ops
    seen = {}

    class Fake:
        def __init__(self, sd, **kw):
            seen.update(kw)

    monkeypatch.setattr(ops, "Encoder", Fake)
    _, ckpt = golden_dataset_small
    VE.load_model(ckpt, compute="f32x3")
    assert (seen["d_model"], seen["time_layers"], seen["time_heads"], seen["compute"]) == (64, 2, 4, "f32")
    from tests.golden.dataset_spec import golden_state_dict
    # a bare state dict takes the reference's defaults (eval.py:139-143), in memory as on disk
    VE.load_model(golden_state_dict("small"), compute="f16")
    assert (seen["d_model"], seen["time_layers"], seen["time_heads"], seen["compute"]) == (256, 4, 8, "f16")
    torch.save({k: torch.as_tensor(np.asarray(v)) for k, v in golden_state_dict("small").items()}, tmp_path / "bare.pt")
    VE.load_model(str(tmp_path / "bare.pt"), compute="f16")
    assert (seen["d_model"], seen["time_layers"], seen["time_heads"], seen["compute"]) == (256, 4, 8, "f16")
    from tests.golden.dataset_spec import SMALL_HP
    VE.load_model((golden_state_dict("small"), dict(SMALL_HP)), compute="f16")
    assert (seen["d_model"], seen["time_layers"], seen["time_heads"], seen["compute"]) == (64, 2, 4, "f32")
    VE.load_model(golden_state_dict("kp"), compute="f16")
    assert (seen["d_model"], seen["time_layers"], seen["compute"]) == (256, 4, "f16")


# ------------------------------------------------------------------------------------------------------ GPU

@pytest.fixture(scope="module")
def vg():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vge import eval as VE
    from vge import ops
    return VE, ops


@gpu
def test_small_checkpoint_embeddings_centroids(vg, golden_dataset_small, golden_flow_small, golden_meta_small):
    VE, ops = vg
    from vge.data import ACTION_CLASSES, NpzVideoDataset, create_dataset_from_generated_meshes, train_test_split
    paths, ckpt = golden_dataset_small
    real_ds = NpzVideoDataset(paths["real"], filter_classes=ACTION_CLASSES)
    train_ds, _ = train_test_split(real_ds, train_ratio=0.8, seed=1337)
    store = ops.DeviceFrameStore.from_host(VE.load_frame_store(train_ds.items, paths["real_kp"], True), DEV)
    stats = VE.compute_stats_from_npz(train_ds.items, paths["real_kp"], device=DEV, store=store)
    raw, diff = VE.infer_dims_from_stats(stats)
    model = VE.load_model(ckpt, raw, diff, device=DEV)
    assert model.compute == "f32" and model.d_model == 64
    ds = create_dataset_from_generated_meshes(paths["generated_meshes"])
    f = VE.extract_window_features(model, ds, paths["generated_kps"], stats, device=DEV, frame_embed=True)
    seq_err = np.abs(f["seq_embeds"].cpu().numpy() - golden_flow_small["seq_embeds"]).max()
    fe_err = np.abs(f["frame_embeds"][:4].cpu().numpy() - golden_flow_small["frame_embeds_first4"]).max()
    print(f"small checkpoint: max |seq - ref| {seq_err:.2e}, max |frame - ref| {fe_err:.2e}")
    assert seq_err < 2e-5 and fe_err < 2e-5
    cents, _, counts = VE.build_real_centroids(model, paths["real"], paths["real_kp"], stats, device=DEV,
                                               train_items=train_ds.items, label_dict=golden_meta_small["label_dict"],
                                               store=store)
    assert np.array_equal(counts.cpu().numpy(), golden_flow_small["counts"])
    assert np.abs(cents.cpu().numpy() - golden_flow_small["centroids"]).max() < 2e-5


@gpu
def test_small_checkpoint_video_scores_match_reference(vg, golden_dataset_small, golden_meta_small, tmp_path):
    """The whole eval.py flow with the d_model 64 / 2-layer / 4-head checkpoint -> video_scores.json within 1e-4."""
    VE, _ = vg
    paths, ckpt = golden_dataset_small
    out = tmp_path / "video_scores.json"
    combined = VE.run_eval(paths["generated_meshes"], paths["real"], ckpt, paths["generated_kps"], paths["real_kp"],
                           out_json=str(out), device=DEV)
    ref = golden_meta_small["video_scores"]
    assert sorted(combined) == sorted(ref)
    for v, e in ref.items():
        assert set(e) == set(combined[v]), v
    worst = max(abs(ref[v][k] - combined[v][k]) for v in ref for k in ref[v])
    print(f"small checkpoint: max |score - reference| = {worst:.2e}")
    assert worst < 1e-4, worst
    assert json.loads(out.read_text()) == combined


@gpu
@pytest.mark.parametrize("compute", ["f32x3", "f16"])
def test_small_checkpoint_tiled_modes_refuse(vg, small_state_dict, compute):
    """The tiled kernels are built for d_model 256 x 8 heads: another shape is VGE_ERR_UNSUPPORTED, never a wrong
    answer (load_model itself routes such checkpoints to f32)."""
    _, ops = vg
    from vge.lib import UnsupportedModelError
    with pytest.raises(UnsupportedModelError):
        ops.Encoder(small_state_dict, time_layers=2, time_heads=4, d_model=64, device=DEV, compute=compute)
