"""Golden file for the per-video npz format, written by the REFERENCE's own save_video_npz (build container only):

    PYTHONDONTWRITEBYTECODE=1 python -B tests/golden/make_npz_format_golden.py

extract_mesh.py imports cv2 and TokenHMR at module level, so this script parses it with ``ast`` and executes only
``mesh_info_to_arrays`` and ``save_video_npz`` (extract_mesh.py:12-43; they need numpy, json and pathlib) on a
small synthetic mesh_info (unsorted frame ids, float64 inputs), and stores the resulting file as
tests/golden/npz_format/Action/v_ref.npz.  Nothing from the reference is copied; the file is its output.
"""
from __future__ import annotations

import ast
import json
import shutil
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
SRC = Path("/root/reference/extract_mesh.py")


def sample_mesh_info():
    rng = np.random.default_rng(7)
    return {int(f): {"pose": rng.standard_normal((23, 3, 3)), "betas": rng.standard_normal(10).astype(np.float32),
                     "global_orient": rng.standard_normal((1, 3, 3)), "vit": rng.standard_normal(16)}
            for f in (4, 0, 2, 7)}


def main():
    tree = ast.parse(SRC.read_text())
    fns = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in ("mesh_info_to_arrays", "save_video_npz")]
    ns = {"np": np, "json": json, "Path": Path}
    exec(compile(ast.Module(body=fns, type_ignores=[]), str(SRC), "exec"), ns)
    out = HERE / "npz_format"
    shutil.rmtree(out, ignore_errors=True)
    p = ns["save_video_npz"]("Action/v_ref", sample_mesh_info(), out_root=str(out),
                             meta={"action": "Action", "video": "v_ref.avi", "source_path": "x/v_ref.avi"})
    print("wrote", p)


if __name__ == "__main__":
    main()
