"""Generate tests/golden/golden_report.json by running the REFERENCE's process_scores.py (build container only).

    PYTHONDONTWRITEBYTECODE=1 python -B tests/golden/make_report_golden.py

process_scores.main() reads static/images/scores.json relative to the working directory and writes
static/images/comparison_table.json next to it; it is run in a scratch directory on each input set below,
and parse_filename on a list of names.  Only the inputs and the reference's outputs are stored.

Input sets (scores are seeded numpy draws, so the file is reproducible):
  tag        every name of TAG_final_human_scores.json (the reference's own fixture, 5 models x 10 actions)
  golden     video_scores.json of the golden eval flow (tests/golden/golden_scores.json)
  edge       names that take the fallback branches: action at offset 0, CamelCase fallback, unparseable,
             trailing numeric model tokens, no .mp4, repeated (model, action) cells, missing cells
  flat       a single video (min == max -> every normalised value is 50)
"""
from __future__ import annotations

import contextlib
import io
import json
import os
import sys
import tempfile
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REF = "/root/reference"

EDGE_NAMES = [
    "BodyWeightSquats_Hunyuan_01_aaaa0001.mp4",       # action at offset 0 -> model = first token
    "Kling_v2_HandStand_03_bbbb0002.mp4",             # no known action -> CamelCase fallback, model = first token
    "kling_v2_handstand_03_bbbb0003.mp4",             # nothing parseable -> skipped
    "Opensora_768_BodyWeightSquats_01_73f1e099.mp4",  # model with an underscore and a numeric token
    "Model_7_12_PushUps_02_cccc0004",                 # trailing numeric tokens dropped, no .mp4
    "Model_7_12_PushUps_05_cccc0005",                 # same cell again
    "Model_7_12_WallPushups_01_cccc0006.mp4",         # WallPushups (not a PushUps hit: case differs)
    "X_TennisSwingThrowDiscus_01_dddd0007.mp4",       # two actions in one token: list order decides
    "Veo3_SoccerJuggling_01_eeee0008.mp4",
    "Veo3_SoccerJuggling_02_eeee0009.mp4",
    "Veo3_HulaHoop_01_eeee0010.mp4",
    "wan21_JumpingJack_04_ffff0011.mp4",
]


def _run_reference(ps, scores: dict) -> dict:
    with tempfile.TemporaryDirectory() as td:
        os.makedirs(os.path.join(td, "static", "images"))
        with open(os.path.join(td, "static", "images", "scores.json"), "w") as f:
            json.dump(scores, f)
        cwd = os.getcwd()
        os.chdir(td)
        try:
            buf = io.StringIO()
            with contextlib.redirect_stdout(buf):
                ps.main()
        finally:
            os.chdir(cwd)
        with open(os.path.join(td, "static", "images", "comparison_table.json")) as f:
            return {"table": json.load(f), "stdout": buf.getvalue()}


def main():
    sys.path.insert(0, REF)
    import process_scores as ps  # noqa

    rng = np.random.default_rng(2024)
    with open(os.path.join(REF, "TAG_final_human_scores.json")) as f:
        tag_names = sorted(json.load(f))
    with open(HERE / "golden_scores.json") as f:
        golden_scores = json.load(f)["video_scores"]

    def draw(names):
        return {n: {"ac": float(rng.uniform(0.0, 1.2)), "tc": float(rng.uniform(0.1, 0.6))} for n in names}

    inputs = {
        "tag": draw(tag_names),
        "golden": {k: v for k, v in golden_scores.items() if "ac" in v and "tc" in v},
        "edge": draw(EDGE_NAMES),
        "flat": draw(["Hunyuan_PullUps_01_00000001.mp4"]),
    }
    out = {"inputs": inputs, "outputs": {k: _run_reference(ps, v) for k, v in inputs.items()}}
    names = tag_names[::7] + EDGE_NAMES + list(golden_scores)[:10]
    out["parse_filename"] = [[n, *ps.parse_filename(n)] for n in names]
    with open(HERE / "golden_report.json", "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", HERE / "golden_report.json")


if __name__ == "__main__":
    main()
