"""ctypes binding of libvge.so (include/vge.h).  The product path has no fallback: if the HIP
library cannot be loaded every compute call raises VgeError."""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

_HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("VGE_LIB", _HERE / "libvge.so"))

VGE_OK = 0
STATUS = {0: "VGE_OK", 1: "VGE_ERR_ARG", 2: "VGE_ERR_HIP", 3: "VGE_ERR_MISSING_WEIGHT", 4: "VGE_ERR_WEIGHT_SHAPE",
          5: "VGE_ERR_NOMEM", 6: "VGE_ERR_WORKSPACE", 7: "VGE_ERR_UNSUPPORTED", 8: "VGE_ERR_DEVICE"}
VGE_ERR_UNSUPPORTED = 7
VGE_ERR_DEVICE = 8

EXPORTS = ["vge_featurize", "vge_featurize_layout", "vge_layout_feat_dim", "vge_stats_finalize_layout",
           "vge_encoder_feat_dim", "vge_stats_workspace_bytes", "vge_stats_accumulate", "vge_stats_finalize",
           "vge_encoder_create", "vge_encoder_reserve", "vge_encoder_destroy", "vge_encode", "vge_tc_windows",
           "vge_score_videos", "vge_centroid_accumulate", "vge_centroid_finalize", "vge_last_error", "vge_version",
           "vge_encoder_profile_begin", "vge_encoder_profile_read", "vge_encoder_profile_mask", "vge_encoder_wait_conv", "vge_ingest_probe",
           "vge_encoder_set_tail_stream", "vge_encoder_status", "vge_encoder_clear_status",
           "vge_ingest_decode",
           "vge_ingest_default_threads",
           "vge_hmr_create", "vge_hmr_reserve", "vge_hmr_destroy", "vge_hmr_extract", "vge_hmr_profile_begin",
           "vge_hmr_profile_read", "vge_op_gemm_bf16", "vge_op_gemm_lib", "vge_op_vit_attention", "vge_op_layernorm_bf16",
           "vge_dwpose_create", "vge_dwpose_reserve", "vge_dwpose_destroy", "vge_dwpose_keypoints",
           "vge_dwpose_profile_begin", "vge_dwpose_profile_read", "vge_op_conv_bf16",
           "vge_yolox_create", "vge_yolox_reserve", "vge_yolox_destroy", "vge_yolox_detect", "vge_yolox_detect_scored",
           "vge_hmr_crop",
           "vge_yolox_profile_begin", "vge_yolox_profile_read",
           "vge_frcnn_create", "vge_frcnn_reserve", "vge_frcnn_destroy", "vge_frcnn_shapes", "vge_frcnn_detect",
           "vge_frcnn_profile_begin", "vge_frcnn_profile_read"]


class VgeError(RuntimeError):
    pass


class UnsupportedModelError(VgeError):
    """VGE_ERR_UNSUPPORTED: a checkpoint whose d_model / time_heads / modality set the kernels are not built for
    (load_model, eval.py:136-165, would build such a HumanActionScorer; this library refuses it by name)."""


class DeviceFaultError(VgeError):
    """VGE_ERR_DEVICE: a kernel raised the encoder's status word (a broken invariant, e.g. the conv kernel's
    half-workgroup exchange wait ran out): the results of that launch are wrong and must not be used."""


class Dims(C.Structure):
    _fields_ = [("n_modalities", C.c_int), ("dims_raw", C.c_int * 8), ("dims_diff", C.c_int * 8),
                ("d_model", C.c_int), ("time_layers", C.c_int), ("time_heads", C.c_int), ("clip_len", C.c_int)]


class TensorView(C.Structure):
    _fields_ = [("name", C.c_char_p), ("data", C.c_void_p), ("ndim", C.c_int), ("shape", C.c_int64 * 4)]


class ClipInfo(C.Structure):  # include/vge_ingest.h vge_clip_info
    _fields_ = [("n_frames", C.c_int32), ("vit_dim", C.c_int32), ("kp_frames", C.c_int32), ("status", C.c_int32)]


INGEST_STATUS = {0: "OK", 1: "ERR_ARG", 7: "ERR_IO", 8: "ERR_SHAPE", 9: "ERR_KP"}


class FrameStoreC(C.Structure):
    _fields_ = [("pose", C.c_void_p), ("gori", C.c_void_p), ("betas", C.c_void_p), ("vit", C.c_void_p),
                ("kp", C.c_void_p), ("videos", C.c_void_p), ("n_videos", C.c_int)]


_lib = None


def load() -> C.CDLL:
    """Load libvge.so once; raise VgeError (no CPU fallback) when it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise VgeError(f"libvge.so not found at {LIB_PATH}: build it with `make -C video-gen-evals_amd/csrc` "
                       "(or __graft_entry__.build()); there is no CPU fallback")
    lib = C.CDLL(str(LIB_PATH))
    vp, i32, i64p = C.c_void_p, C.c_int, C.POINTER(C.c_int64)
    sig = {
        "vge_featurize": [C.POINTER(FrameStoreC), vp, i32, vp, vp, vp, vp],
        "vge_featurize_layout": [C.POINTER(FrameStoreC), vp, i32, vp, vp, i32, vp, vp],
        "vge_layout_feat_dim": [i32],
        "vge_stats_finalize_layout": [vp, i64p, i32, vp, vp, vp],
        "vge_encoder_feat_dim": [vp],
        "vge_stats_workspace_bytes": [i32],
        "vge_stats_accumulate": [C.POINTER(FrameStoreC), vp, vp, i32, vp, i64p, vp, C.c_size_t, vp],
        "vge_stats_finalize": [vp, i64p, vp, vp, vp],
        "vge_encoder_create": [C.POINTER(Dims), C.POINTER(TensorView), i32, i32, C.POINTER(vp)],
        "vge_encoder_reserve": [vp, i32],
        "vge_encoder_destroy": [vp],
        "vge_encode": [vp, vp, i32, i32, vp, vp, vp, vp],
        "vge_tc_windows": [vp, i32, i32, i32, vp, vp],
        "vge_score_videos": [vp, vp, vp, vp, vp, i32, i32, vp, vp, vp],
        "vge_centroid_accumulate": [vp, vp, i32, i32, i32, vp, vp, vp],
        "vge_centroid_finalize": [vp, vp, i32, i32, vp, vp],
        "vge_encoder_profile_begin": [vp, i32],
        "vge_encoder_wait_conv": [vp, vp],
        "vge_encoder_set_tail_stream": [vp, vp],
        "vge_encoder_profile_mask": [vp, i32],
        "vge_encoder_profile_read": [vp, C.POINTER(C.c_double), C.POINTER(C.c_int)],
        "vge_encoder_status": [vp],
        "vge_encoder_clear_status": [vp],
        "vge_last_error": [],
        "vge_version": [],
        "vge_ingest_probe": [C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), i32, i32, C.POINTER(ClipInfo)],
        "vge_ingest_decode": [C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), i32, i32, vp, i32, vp, vp, vp, vp, vp,
                              vp],
    }
    for name, args in sig.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = C.c_int
    lib.vge_stats_workspace_bytes.restype = C.c_size_t
    lib.vge_last_error.restype = C.c_char_p
    lib.vge_version.restype = C.c_char_p
    _lib = lib
    return lib


def check(status: int, what: str) -> None:
    if status != VGE_OK:
        msg = load().vge_last_error().decode(errors="replace")
        cls = {VGE_ERR_UNSUPPORTED: UnsupportedModelError, VGE_ERR_DEVICE: DeviceFaultError}.get(status, VgeError)
        raise cls(f"{what} failed: {STATUS.get(status, status)}: {msg}")
