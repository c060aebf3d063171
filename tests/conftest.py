import json
import os
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "video-gen-evals_amd"))
sys.path.insert(0, str(REPO))

GOLDEN = REPO / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libvge.so on cuda:0)")


@pytest.fixture(scope="session")
def golden_dataset(tmp_path_factory):
    """The synthetic dataset + checkpoint the golden vectors were generated from."""
    from tests.golden.dataset_spec import build_golden_dataset
    root = tmp_path_factory.mktemp("golden_ds")
    paths, ckpt, digest = build_golden_dataset(str(root))
    flow = np.load(GOLDEN / "golden_flow.npz")
    assert bytes(flow["dataset_digest"]).hex() == digest, "synthetic generator drifted from the golden fixtures"
    return paths, ckpt


@pytest.fixture(scope="session")
def golden_flow():
    return dict(np.load(GOLDEN / "golden_flow.npz"))


@pytest.fixture(scope="session")
def golden_meta():
    with open(GOLDEN / "golden_scores.json") as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_ops():
    return dict(np.load(GOLDEN / "golden_ops.npz"))


@pytest.fixture(scope="session")
def golden_state_dict():
    from vge import synth
    return synth.make_state_dict(synth.DIMS_RAW, synth.DIMS_DIFF)


# ---- the keypoint-less flow (keypoint_dir None: 4 modalities, feats rows of 2356)

@pytest.fixture(scope="session")
def golden_dataset_nokp(tmp_path_factory):
    from tests.golden.dataset_spec import build_golden_dataset
    root = tmp_path_factory.mktemp("golden_ds_nokp")
    paths, ckpt, digest = build_golden_dataset(str(root), layout="nokp")
    flow = np.load(GOLDEN / "golden_flow_nokp.npz")
    assert bytes(flow["dataset_digest"]).hex() == digest, "synthetic generator drifted from the golden fixtures"
    return paths, ckpt


@pytest.fixture(scope="session")
def golden_flow_nokp():
    return dict(np.load(GOLDEN / "golden_flow_nokp.npz"))


@pytest.fixture(scope="session")
def golden_meta_nokp():
    with open(GOLDEN / "golden_scores_nokp.json") as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_state_dict_nokp():
    from tests.golden.dataset_spec import golden_state_dict
    return golden_state_dict("nokp")


# ---- a checkpoint of another shape (d_model 64, 2 layers, 4 heads: dataset_spec.SMALL_HP)

@pytest.fixture(scope="session")
def golden_dataset_small(tmp_path_factory):
    from tests.golden.dataset_spec import build_golden_dataset
    root = tmp_path_factory.mktemp("golden_ds_small")
    paths, ckpt, digest = build_golden_dataset(str(root), layout="small")
    flow = np.load(GOLDEN / "golden_flow_small.npz")
    assert bytes(flow["dataset_digest"]).hex() == digest, "synthetic generator drifted from the golden fixtures"
    return paths, ckpt


@pytest.fixture(scope="session")
def golden_flow_small():
    return dict(np.load(GOLDEN / "golden_flow_small.npz"))


@pytest.fixture(scope="session")
def golden_meta_small():
    with open(GOLDEN / "golden_scores_small.json") as f:
        return json.load(f)
