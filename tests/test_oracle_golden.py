"""Pin the oracle (CPU restatement) against golden vectors produced by the reference itself."""
import numpy as np
import pytest
import torch

from oracle import featurize as OF
from oracle.lapack2x2 import sgesdd_2x2


def test_svd2x2_lapack_signs():
    from tests.conftest import GOLDEN
    z = np.load(GOLDEN / "svd2x2.npz")
    U, S, Vh = sgesdd_2x2(z["H"])
    assert np.abs(U - z["U"]).max() < 2e-6
    assert np.abs(Vh - z["Vh"]).max() < 2e-6
    assert np.abs(S - z["S"]).max() < 2e-6


def test_rotmat_delta(golden_ops):
    for k in ("rot", "rotnear"):
        got = OF.rotmat_delta(golden_ops[k + "_in"])
        # the log map is ill-conditioned near theta = pi (1/sin theta): 1e-4 on angles up to pi
        assert np.abs(got - golden_ops[k + "_delta"]).max() < 1e-4, k
    got = OF.log_so3(golden_ops["logso3_in"])
    assert np.abs(got - golden_ops["logso3_out"]).max() < 2e-5


def test_vit_beta_delta(golden_ops):
    assert np.abs(OF.vit_delta(golden_ops["vit_in"]) - golden_ops["vit_delta"]).max() < 1e-6
    assert np.array_equal(OF.betas_delta(golden_ops["beta_in"]), golden_ops["beta_delta"])


@pytest.mark.parametrize("name", ["kp_rand", "kp_static", "kp_neg", "kp_mixed"])
def test_procrustes(golden_ops, name):
    got = OF.procrustes_kp_delta(golden_ops[name + "_in"])
    assert np.abs(got - golden_ops[name + "_delta"]).max() < 2e-5, name


def _both_branches(kp):
    """Per-frame deltas for the two admissible signs of the null-space singular vector."""
    T = kp.shape[0]
    pts = kp.reshape(T, -1, 2).astype(np.float64)
    pc = pts - pts.mean(1, keepdims=True)
    pn = pc / np.maximum(np.sqrt((pc ** 2).sum((1, 2), keepdims=True)), 1e-6)
    out = []
    for t in range(1, T):
        X, Y = pn[t - 1], pn[t]
        U, _, Vh = np.linalg.svd(X.T @ Y)
        cands = []
        for fu in (1.0, -1.0):
            for fv in (1.0, -1.0):
                U2 = U.copy()
                U2[:, 1] *= fu
                V2 = Vh.copy()
                V2[1, :] *= fv
                R = V2 @ U2.T
                if np.linalg.det(R) < 0:
                    V2[:, -1] *= -1
                    R = V2 @ U2.T
                cands.append((Y - X @ R).reshape(-1))
        out.append(cands)
    return out


def test_procrustes_collinear_degenerate(golden_ops):
    """Exactly collinear keypoints give a rank-1 H: which of two reflections the reference applies
    depends on MKL's float rounding of H (parity unpinned by construction).  Both the reference and
    the oracle must pick one of the two admissible branches on every frame."""
    kp = golden_ops["kp_col_in"]
    got = OF.procrustes_kp_delta(kp)
    ref = golden_ops["kp_col_delta"]
    for t, cands in enumerate(_both_branches(kp), start=1):
        assert min(np.abs(ref[t] - c).max() for c in cands) < 1e-4, t
        assert min(np.abs(got[t] - c).max() for c in cands) < 1e-4, t


@pytest.mark.parametrize("s", [0, 5, 19, 25, -1])
def test_slice_or_pad(golden_ops, s):
    assert np.array_equal(OF.slice_or_pad(golden_ops["sop_in"], s, 32), golden_ops[f"sop_{s}"])


@pytest.fixture(scope="module")
def oracle_run(golden_dataset, golden_state_dict, golden_meta):
    from oracle import evalflow
    paths, _ = golden_dataset
    return evalflow.run_eval(paths["real"], paths["real_kp"], paths["generated_meshes"], paths["generated_kps"],
                             golden_state_dict, dict(golden_meta["dims_raw"]), dict(golden_meta["dims_diff"]))


def test_oracle_stats(oracle_run, golden_flow):
    _, ex = oracle_run
    mean, std = ex["stats"].concat()
    assert np.abs(mean - golden_flow["stats_mean"]).max() < 1e-6
    assert np.abs(std - golden_flow["stats_std"]).max() < 1e-6


def test_oracle_centroids(oracle_run, golden_flow, golden_meta):
    _, ex = oracle_run
    assert ex["label_dict"] == golden_meta["label_dict"]
    assert np.array_equal(ex["counts"].numpy(), golden_flow["counts"])
    assert np.abs(ex["centroids"].numpy() - golden_flow["centroids"]).max() < 1e-5


def test_oracle_embeddings(oracle_run, golden_flow):
    _, ex = oracle_run
    assert np.abs(ex["seq"].numpy() - golden_flow["seq_embeds"]).max() < 1e-5
    assert np.abs(ex["frame_embeds"][:4].numpy() - golden_flow["frame_embeds_first4"]).max() < 1e-5


def test_oracle_feats(golden_dataset, golden_flow, golden_meta, oracle_run):
    from oracle import evalflow
    paths, _ = golden_dataset
    _, ex = oracle_run
    items = evalflow.scan_generated(paths["generated_meshes"])
    samples = [(c, n, p, s) for c, n, p, T in items for s in evalflow.windows_for(T)]
    for wi, ref in zip(golden_flow["feat_windows"], golden_flow["feats_sel"]):
        c, n, p, s = samples[wi]
        pose, gori, betas, vit, kp = evalflow.load(p, paths["generated_kps"], c)
        got = OF.featurize_window(pose, gori, betas, vit, kp, s, ex["stats"])
        assert np.abs(got - ref).max() < 1e-4, (wi, np.abs(got - ref).max())


def test_oracle_scores(oracle_run, golden_meta):
    combined, _ = oracle_run
    ref = golden_meta["video_scores"]
    assert sorted(combined) == sorted(ref)
    for v, e in ref.items():
        assert set(e) == set(combined[v]), v
        for k in e:
            assert abs(e[k] - combined[v][k]) < 1e-5, (v, k)
