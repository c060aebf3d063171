"""The C-ABI library loads and exports every entry point include/vge.h declares (no GPU needed)."""
import re
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent


def declared():
    txt = (REPO / "include" / "vge.h").read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(vge_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_expected_entry_points():
    names = declared()
    for must in ("vge_featurize", "vge_encode", "vge_encoder_create", "vge_score_videos", "vge_centroid_accumulate",
                 "vge_stats_accumulate", "vge_tc_windows"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from vge import lib as L
    if not L.LIB_PATH.exists():
        pytest.fail(f"{L.LIB_PATH} missing: run __graft_entry__.build()")
    so = L.load()
    for name in declared():
        assert hasattr(so, name), name
    assert set(L.EXPORTS) == set(declared())
    assert b"gfx950" in so.vge_version()


def test_error_path_without_gpu_work():
    """Argument errors are reported through status codes + vge_last_error, never exceptions."""
    import ctypes as C
    from vge import lib as L
    so = L.load()
    st = so.vge_featurize(None, None, 0, None, None, None, None)
    assert st == 1
    assert b"vge_featurize" in so.vge_last_error()
    h = C.c_void_p()
    dims = L.Dims()
    assert so.vge_encoder_create(C.byref(dims), None, 0, 0, C.byref(h)) == 1
