"""The C-ABI library loads and exports every entry point include/vge.h declares (no GPU needed)."""
import re
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent


def declared():
    txt = "\n".join(h.read_text() for h in sorted((REPO / "include").glob("*.h")))
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
    assert so.vge_encoder_wait_conv(None, None) == 1
    assert b"vge_encoder_wait_conv" in so.vge_last_error()
    assert so.vge_encoder_set_tail_stream(None, None) == 1
    assert b"vge_encoder_set_tail_stream" in so.vge_last_error()
    assert so.vge_encoder_status(None) == 1 and b"vge_encoder_status" in so.vge_last_error()
    assert so.vge_encoder_clear_status(None) == 1


def test_device_status_is_plumbed_to_its_own_error():
    """The conv kernel's status word (raised when its exchange wait runs out) reaches Python as DeviceFaultError:
    the header declares VGE_ERR_DEVICE = 8, the binding maps that code to its own exception class, and the kernel's
    spin-bound hook is exported (the GPU test forces the bound to 0 and checks the error)."""
    import re as _re
    from vge import lib as L
    hdr = (REPO / "include" / "vge.h").read_text()
    assert _re.search(r"VGE_ERR_DEVICE\s*=\s*8", hdr)
    assert L.STATUS[8] == "VGE_ERR_DEVICE" and L.VGE_ERR_DEVICE == 8
    so = L.load()
    assert hasattr(so, "vge_debug_set_x3s_spin_limit")
    prev = so.vge_debug_set_x3s_spin_limit(5)
    assert so.vge_debug_set_x3s_spin_limit(-1) == 5
    assert so.vge_debug_set_x3s_spin_limit(-1) == prev == (1 << 22)
    orig = so.vge_last_error
    try:
        so.vge_last_error = lambda: b"status word set"
        with pytest.raises(L.DeviceFaultError, match="VGE_ERR_DEVICE"):
            L.check(L.VGE_ERR_DEVICE, "vge_encode")
    finally:
        so.vge_last_error = orig


def _hexf(s):
    return float.fromhex(s)


def test_erf_branch_free_accuracy():
    """Host restatement (float32 numpy) of the device GELU's branch-free erf (vge_common.h gelu2_many): the
    ocml erff minimax pieces, both evaluated and selected.  |error| vs math.erf stays at f32 rounding level."""
    import math
    import numpy as np
    f = np.float32
    c = [f(_hexf(x)) for x in ("-0x1.268bc2p-11", "0x1.420828p-8", "-0x1.b5937p-6", "0x1.ce077cp-4",
                               "-0x1.81266p-2", "0x1.06eba0p-3")]
    d = [f(_hexf(x)) for x in ("0x1.1d3156p-16", "-0x1.8d129p-12", "0x1.f9a6d2p-9", "-0x1.8c3164p-6",
                               "0x1.b4e9c8p-4", "0x1.4515fap-1", "0x1.078e5p-3")]
    z = np.linspace(-6, 6, 200001, dtype=np.float32)
    a = np.abs(z)
    s = a * a
    q = s * c[0] + c[1]
    for k in c[2:]:
        q = s * q + k
    small = a * q + a
    p = a * d[0] + d[1]
    for k in d[2:]:
        p = a * p + k
    p = a * p + a
    big = f(1) - np.exp2(p * f(-1.44269504))
    erf = np.copysign(np.where(a < 1, small, big), z)
    ref = np.array([math.erf(float(v)) for v in z])
    assert np.abs(erf - ref).max() < 1.5e-7


def test_gelu_fast_accuracy():
    """Host restatement (float32 numpy) of the fp16 conv path's GELU (vge_common.h gelu2_fast): erf(|x|/sqrt 2) =
    1 - 2^(-a P(a)), a = min(|x|, 4 sqrt 2), GELU = 0.5 x + |x| (0.5 - 0.5 * 2^(-a P(a))).  |error| vs the exact
    GELU stays below 5e-7 over [-10, 10] (that path's operands are fp16: 2^-11 relative)."""
    import math
    import numpy as np
    f = np.float32
    c = [f(_hexf(x)) for x in ("-0x1.f5fbdcp-16", "0x1.83e48ap-11", "-0x1.05672ep-7", "0x1.b42062p-5",
                               "0x1.d5ee02p-2", "0x1.26b194p+0")]
    x = np.linspace(-10, 10, 400001, dtype=np.float32)
    a = np.minimum(np.abs(x), f(_hexf("0x1.6a09e6p+2")))
    p = a * c[0] + c[1]
    for k in c[2:]:
        p = a * p + k
    p = p * a
    eh = np.exp2(-p.astype(np.float64)).astype(np.float32) * f(-0.5) + f(0.5)
    out = np.abs(x) * eh + x * f(0.5)
    ref = np.array([0.5 * float(v) * (1 + math.erf(float(v) / math.sqrt(2))) for v in x])
    assert np.abs(out - ref).max() < 5e-7


@pytest.mark.parametrize("field,value", [("d_model", 128), ("time_heads", 4), ("n_modalities", 6), ("n_modalities", 3),
                                         ("clip_len", 64)])
def test_unsupported_model_shape_has_its_own_status(field, value):
    """load_model (eval.py:136-165) builds HumanActionScorer with d_model / time_layers / time_heads from the
    checkpoint; the modality set is the five of the keypoint layout or the keypoint-less four (utils.py:496-514),
    clip / dino modalities (6 / 7) are not built.  Shapes the kernels are not built for are refused before any
    device work with VGE_ERR_UNSUPPORTED (UnsupportedModelError in Python), distinct from argument errors;
    time_layers is free."""
    import ctypes as C
    from vge import lib as L
    from vge import ops
    so = L.load()
    dims = L.Dims()
    dims.n_modalities, dims.d_model, dims.time_layers, dims.time_heads, dims.clip_len = 5, 256, 4, 8, 32
    for i in range(5):
        dims.dims_raw[i], dims.dims_diff[i] = ops.DIMS_RAW[i], ops.DIMS_DIFF[i]
    setattr(dims, field, value)
    h = C.c_void_p()
    st = so.vge_encoder_create(C.byref(dims), (L.TensorView * 1)(), 0, 1, C.byref(h))
    assert st == L.VGE_ERR_UNSUPPORTED, st
    with pytest.raises(L.UnsupportedModelError, match="VGE_ERR_UNSUPPORTED"):
        L.check(st, "vge_encoder_create")
    dims.time_layers = 0
    setattr(dims, field, {"d_model": 256, "time_heads": 8, "n_modalities": 5, "clip_len": 32}[field])
    assert so.vge_encoder_create(C.byref(dims), (L.TensorView * 1)(), 0, 1, C.byref(h)) == 1  # VGE_ERR_ARG


@pytest.mark.parametrize("d_model,heads,expect", [(128, 4, "missing"), (64, 4, "missing"), (96, 1, "unsupported"),
                                                   (320, 8, "unsupported"), (80, 8, "unsupported"), (256, 2, "unsupported")])
def test_generic_f32_shapes(d_model, heads, expect):
    """VGE_F32 takes other checkpoint shapes on the generic kernels (d_model a multiple of 32 in [32, 256], head dim
    <= 64): such a create gets past the shape check to the weights (an empty list: VGE_ERR_MISSING_WEIGHT); others
    stay VGE_ERR_UNSUPPORTED.  No device work happens before the weights are complete."""
    import ctypes as C
    from vge import lib as L
    from vge import ops
    so = L.load()
    dims = L.Dims()
    dims.n_modalities, dims.d_model, dims.time_layers, dims.time_heads, dims.clip_len = 5, d_model, 2, heads, 32
    for i in range(5):
        dims.dims_raw[i], dims.dims_diff[i] = ops.DIMS_RAW[i], ops.DIMS_DIFF[i]
    h = C.c_void_p()
    st = so.vge_encoder_create(C.byref(dims), (L.TensorView * 1)(), 0, 0, C.byref(h))
    assert st == (L.VGE_ERR_UNSUPPORTED if expect == "unsupported" else 3), st


def test_load_model_refuses_clip_modality():
    """The keypoint-less four are built (tests/test_nokp_layout.py); a CLIP-embedding modality is not."""
    from vge import eval as VE
    from vge.lib import UnsupportedModelError
    raw = {"vit": 1024, "global": 9, "pose": 207, "beta": 10, "kp2d": 120, "clip": 512}
    diff = {"vit": 1024, "global": 3, "pose": 69, "beta": 10, "kp2d": 120, "clip": 512}
    with pytest.raises(UnsupportedModelError):
        VE.load_model({}, raw, diff, device="cpu")


@pytest.mark.parametrize("n_windows", [1, 3, 37, 64, 255, 256, 293, 512, 600, 4096])
def test_conv_unit_schedule_covers_every_window_once(n_windows):
    """Host-side unit table of the fp16 conv kernel (vge_encoder_x3.hip conv_f16w_schedule, host only, 256 CUs
    assumed without a GPU): every (encoder, window) pair in exactly one unit of 1..6 consecutive windows; the fewest
    rounds; per-CU windows within one unit of balance.  At the bench's 256 windows: two units per CU (quint + quint
    or hex + quad), 10 windows each."""
    import collections
    import ctypes as C

    import numpy as np
    from vge import lib as L
    so = L.load()
    cap = 10 * n_windows + 1024
    tab = np.zeros(cap, np.int32)
    G, R = C.c_int(), C.c_int()
    n = so.vge_debug_conv_schedule(n_windows, 6, tab.ctypes.data_as(C.c_void_p), cap, C.byref(G), C.byref(R))
    assert n == G.value * R.value > 0
    tab = tab[:n].reshape(R.value, G.value)
    seen = collections.Counter()
    per_cu = np.zeros(G.value, np.int64)
    for u in tab.ravel():
        if u < 0:
            continue
        e, w, w0 = u & 15, (u >> 4) & 7, u >> 8
        assert 1 <= w <= 6 and 0 <= w0 and w0 + w <= n_windows and e < 10
        for k in range(w0, w0 + w):
            seen[(e, k)] += 1
    for r in range(R.value):
        for p in range(G.value):
            if tab[r, p] >= 0:
                per_cu[p] += (tab[r, p] >> 4) & 7
    assert len(seen) == 10 * n_windows and set(seen.values()) == {1}
    assert per_cu.max() - per_cu.min() <= 6
    if n_windows == 256:
        assert (G.value, R.value) == (256, 2) and set(per_cu.tolist()) == {10}


@pytest.mark.parametrize("heavy", [False, True])
@pytest.mark.parametrize("n_enc", [10, 8])
@pytest.mark.parametrize("n_windows", [1, 2, 3, 5, 37, 64, 255, 256, 293, 512, 600, 4096])
def test_quad_schedule_covers_every_window_once(n_windows, n_enc, heavy):
    """Quad / pair schedule of the split-precision conv kernels (conv_quad_sched + conv_unit, as the kernels decode it;
    256 CUs assumed without a GPU): every (encoder, window) pair in exactly one unit, quads in the rounds before the
    pairs, every CU within one quad of the others.  At the bench's 256 windows every XCD's run of 32 CUs works on ONE
    encoder in each round (24 encoder weight streams per launch; vge_x3.h), and with the vit encoders marked heavy
    (multi-panel stems) every CU runs exactly one vit unit, a pair."""
    import collections
    import ctypes as C

    import numpy as np
    from vge import lib as L
    so = L.load()
    cap = 3 * (10 * n_windows + 1024)
    tab = np.zeros(cap, np.int32)
    G = C.c_int()
    hv = ({10: 0x21, 8: 0x11}[n_enc]) if heavy else 0  # state / motion vit (vge/eval.py modality order)
    n = so.vge_debug_quad_schedule(n_windows, n_enc, hv, tab.ctypes.data_as(C.c_void_p), cap // 3, C.byref(G))
    assert n > 0 and n % G.value == 0
    tab = tab[:3 * n].reshape(n // G.value, G.value, 3)
    seen = collections.Counter()
    per_cu = np.zeros(G.value, np.int64)
    for r in range(tab.shape[0]):
        for p in range(G.value):
            e, w0, w = tab[r, p]
            if w < 0:
                continue
            assert w in (2, 4) and 0 <= e < n_enc and w0 % 2 == 0 and 0 <= w0 < n_windows
            if w == 4:
                assert w0 + 4 <= n_windows
            for k in range(w0, min(w0 + w, n_windows)):  # a pair may be half past the end (odd n_windows)
                seen[(e, k)] += 1
            per_cu[p] += w
    assert len(seen) == n_enc * n_windows and set(seen.values()) == {1}
    assert per_cu.max() - per_cu.min() <= 4
    if n_windows == 256:
        streams = 0
        for r in range(tab.shape[0]):
            for x in range(8):
                run = tab[r, x::8]  # blocks of XCD x (dealt round robin), in xcd_remap order
                streams += len({int(e) for e, _, w in run if w > 0})
        assert streams == {10: 24, 8: 16}[n_enc]
        if heavy and n_enc == 10:
            assert tab.shape[0] == 3
            for p in range(G.value):
                units = [tuple(tab[r, p]) for r in range(3)]
                assert [w for _, _, w in units] == [4, 4, 2]
                assert sum((hv >> e) & 1 for e, _, _ in units) == 1 and (hv >> units[2][0]) & 1
