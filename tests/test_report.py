"""Post-hoc reporting against fixtures produced by the reference itself:
the process_scores.py comparison table (tests/golden/golden_report.json, make_report_golden.py) and the
sign-inverted Spearman of eval.py:297-347 (golden_scores.json "spearman", make_golden.py) on the reference's
own TAG_final_human_scores.json (copied to tests/golden/tag_human_scores.json as a data fixture)."""
import contextlib
import io
import json

import pytest

from tests.conftest import GOLDEN
from vge import report


@pytest.fixture(scope="module")
def golden_report():
    with open(GOLDEN / "golden_report.json") as f:
        return json.load(f)


def test_parse_filename(golden_report):
    for name, model, action in golden_report["parse_filename"]:
        assert report.parse_filename(name) == (model, action), name


@pytest.mark.parametrize("case", ["tag", "golden", "edge", "flat"])
def test_comparison_table(golden_report, case):
    scores = golden_report["inputs"][case]
    got = report.comparison_table(scores, log=lambda s: None)
    # exact: same float operations in the same order as the reference, then round()
    assert json.loads(json.dumps(got)) == golden_report["outputs"][case]["table"]


@pytest.mark.parametrize("case", ["edge", "tag"])
def test_cli_output(golden_report, case, tmp_path, monkeypatch):
    """The CLI reads/writes the reference's default paths and prints the same report."""
    (tmp_path / "static" / "images").mkdir(parents=True)
    (tmp_path / "static" / "images" / "scores.json").write_text(json.dumps(golden_report["inputs"][case]))
    monkeypatch.chdir(tmp_path)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        assert report.main([]) == 0
    assert buf.getvalue() == golden_report["outputs"][case]["stdout"]
    written = json.loads((tmp_path / "static" / "images" / "comparison_table.json").read_text())
    assert written == golden_report["outputs"][case]["table"]


def test_missing_scores_file(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    assert report.main([]) == 1


def test_empty_scores_raise():
    with pytest.raises(ValueError):  # min() of no scores, as in the reference
        report.comparison_table({}, log=lambda s: None)


def test_spearman_vs_reference(golden_meta):
    from vge.eval import compute_spearman_correlation
    for key in ("ac", "tc"):
        corr, p, matched = compute_spearman_correlation(golden_meta["spearman_model_scores"],
                                                        str(GOLDEN / "tag_human_scores.json"), key)
        ref = golden_meta["spearman"][key]
        assert len(matched) == ref["n_matched"]
        assert corr == pytest.approx(ref["corr"], abs=1e-12)
        assert p == pytest.approx(ref["p"], rel=1e-9)


def test_spearman_too_few_matches(tmp_path):
    from vge.eval import compute_spearman_correlation
    human = tmp_path / "h.json"
    human.write_text(json.dumps({"A_PushUps_01_x.mp4": {"ac": 1.0}, "B_PushUps_02_y.mp4": {"tc": 2.0}}))
    corr, p, matched = compute_spearman_correlation({"A_PushUps_01_x": 0.3}, str(human), "ac")
    assert corr is None and p is None and len(matched) == 1
