"""Golden vectors for the keypoints.npy row composition, produced by the REFERENCE's own function (build
container only):

    PYTHONDONTWRITEBYTECODE=1 python -B tests/golden/make_kp120_golden.py

modifications/process_video.py cannot be imported here (it imports cv2 and instantiates DWposeDetector at module
level), so this script parses it with ``ast`` and executes only ``flatten_first_person_no_padding``
(process_video.py:23-57), which needs nothing but numpy, on synthetic inputs shaped exactly like
DWposeDetector.__call__'s outputs (dwpose_init.py:44-67: bodies['candidate'] = [nums * 18, 2], hands =
vstack(candidate[:, 92:113], candidate[:, 113:]) = [2 * nums, 21, 2]) plus the malformed shapes the function
guards against.  Stores inputs and outputs in kp120_flatten.npz; nothing from the reference is copied.
"""
from __future__ import annotations

import ast
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
SRC = Path("/root/reference/modifications/process_video.py")


def load_reference_flatten():
    tree = ast.parse(SRC.read_text())
    fn = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "flatten_first_person_no_padding")
    ns = {"np": np}
    exec(compile(ast.Module(body=[fn], type_ignores=[]), str(SRC), "exec"), ns)
    return ns["flatten_first_person_no_padding"]


def main():
    flatten = load_reference_flatten()
    rng = np.random.default_rng(120)
    cases = []
    for nums in (1, 1, 2, 2, 3, 4):  # DWposeDetector-shaped outputs
        cand = rng.random((nums, 134, 2))
        cand[rng.random((nums, 134)) < 0.1] = -1
        body = cand[:, :18].reshape(nums * 18, 2)
        hands = np.vstack([cand[:, 92:113], cand[:, 113:]])
        cases.append(("detector", nums, body, hands))
    one = rng.random((1, 134, 2))
    cases.append(("hands4d", 1, one[:, :18].reshape(18, 2), rng.random((2, 2, 21, 2))))       # (k, 2, 21, 2)
    cases.append(("one_hand", 1, one[:, :18].reshape(18, 2), rng.random((1, 21, 2))))          # -> None
    cases.append(("no_hands", 1, one[:, :18].reshape(18, 2), None))                           # -> None
    cases.append(("short_body", 1, one[:, :10].reshape(10, 2), rng.random((2, 21, 2))))        # -> None
    cases.append(("empty_body", 0, np.zeros((0, 2)), rng.random((2, 21, 2))))                  # -> None
    out = {}
    for i, (kind, nums, body, hands) in enumerate(cases):
        r = flatten({"candidate": body, "subset": None}, hands)
        out[f"c{i}_kind"] = np.array(kind)
        out[f"c{i}_body"] = body
        out[f"c{i}_hands"] = np.zeros((0,)) if hands is None else np.asarray(hands)
        out[f"c{i}_hands_none"] = np.array(hands is None)
        out[f"c{i}_out"] = np.zeros((0,)) if r is None else np.asarray(r)
        out[f"c{i}_none"] = np.array(r is None)
    out["n_cases"] = np.array(len(cases))
    np.savez(HERE / "kp120_flatten.npz", **out)
    print("wrote", HERE / "kp120_flatten.npz", len(cases), "cases")


if __name__ == "__main__":
    main()
