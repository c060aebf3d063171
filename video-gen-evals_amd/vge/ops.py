"""Torch-facing wrappers over libvge.so.  torch supplies device memory and the current HIP stream;
all arithmetic happens in the HIP kernels behind the C ABI (vge.lib)."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, Optional, Sequence, Tuple

import numpy as np
import torch

from . import lib as L
from .data import FrameStore

FEAT_DIM = 2596
D_MODEL = 256
MODALITIES = ("vit", "global", "pose", "beta", "kp2d")
DIMS_RAW = (1024, 9, 207, 10, 120)
DIMS_DIFF = (1024, 3, 69, 10, 120)
# Feature layouts (utils.py:496-514): "kp" when the reference runs with a keypoint_dir (5 modalities, rows of 2596),
# "nokp" when keypoint_dir is None (no kp2d columns: 4 modalities, rows of 2356)
LAYOUTS = {"kp": 0, "nokp": 1}
FEAT_DIMS = {"kp": 2596, "nokp": 2356}
N_MODALITIES = {"kp": 5, "nokp": 4}


def layout_of(keypoint_dir) -> str:
    """The feats layout the reference builds for a keypoint directory (None -> keypoint-less)."""
    return "kp" if keypoint_dir is not None else "nokp"


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    if t is None:
        return None
    if not t.is_cuda:
        raise L.VgeError("vge ops need device (cuda/HIP) tensors")
    if not t.is_contiguous():
        raise L.VgeError("vge ops need contiguous tensors")
    return t.data_ptr()


def _stream(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


@dataclass
class DeviceFrameStore:
    """The frame store resident in HBM (see vge.data.FrameStore) + its C view."""
    pose: torch.Tensor
    gori: torch.Tensor
    betas: torch.Tensor
    vit: torch.Tensor
    kp: torch.Tensor
    videos: torch.Tensor            # int32 [V,4] on device
    host_videos: np.ndarray         # int32 [V,4]
    names: list
    classes: list

    @classmethod
    def from_host(cls, st: FrameStore, device) -> "DeviceFrameStore":
        def dev(a, dtype=torch.float32):
            return torch.from_numpy(np.ascontiguousarray(a)).to(device=device, dtype=dtype)
        return cls(pose=dev(st.pose), gori=dev(st.gori), betas=dev(st.betas), vit=dev(st.vit), kp=dev(st.kp),
                   videos=dev(st.videos, torch.int32), host_videos=np.ascontiguousarray(st.videos, np.int32),
                   names=list(st.names), classes=list(st.classes))

    @property
    def n_videos(self) -> int:
        return int(self.host_videos.shape[0])

    def cview(self) -> L.FrameStoreC:
        return L.FrameStoreC(_ptr(self.pose), _ptr(self.gori), _ptr(self.betas), _ptr(self.vit), _ptr(self.kp),
                             _ptr(self.videos), self.n_videos)


def featurize(store: DeviceFrameStore, windows: torch.Tensor, mean: torch.Tensor, std: torch.Tensor,
              out: Optional[torch.Tensor] = None, layout: str = "kp") -> torch.Tensor:
    """WindowDataset._try_one for a batch of windows -> feats [Nw,32,2596] (utils.py:383-516); layout "nokp"
    (keypoint_dir None): feats [Nw,32,2356] and mean/std [2356] in that layout."""
    lib = L.load()
    n = int(windows.shape[0])
    D = FEAT_DIMS[layout]
    if mean.numel() != D or std.numel() != D:
        raise L.VgeError(f"featurize: mean/std must have {D} entries for layout {layout!r}")
    if out is None:
        out = torch.empty((n, 32, D), device=windows.device, dtype=torch.float32)
    elif tuple(out.shape[1:]) != (32, D) or out.shape[0] < n:
        raise L.VgeError(f"featurize: out must be [>= {n}, 32, {D}] for layout {layout!r}")
    if n:
        cv = store.cview()
        L.check(lib.vge_featurize_layout(C.byref(cv), _ptr(windows), n, _ptr(mean), _ptr(std), LAYOUTS[layout],
                                         _ptr(out), _stream(windows.device)), "vge_featurize")
    return out


def stats_accumulate(store: DeviceFrameStore, video_sel: Sequence[int], sums: torch.Tensor, counts: np.ndarray,
                     workspace_tiles: int = 512) -> None:
    """compute_stats_from_npz's float64 sum / sum-of-squares (utils.py:595-744), accumulated into
    sums [2,2596] f64 (device) and counts int64[2] (host)."""
    lib = L.load()
    sel = np.ascontiguousarray(np.asarray(video_sel, np.int32))
    wsb = lib.vge_stats_workspace_bytes(workspace_tiles)
    ws = torch.empty(wsb, dtype=torch.uint8, device=sums.device)
    cnt = (C.c_int64 * 2)(int(counts[0]), int(counts[1]))
    cv = store.cview()
    L.check(lib.vge_stats_accumulate(C.byref(cv), store.host_videos.ctypes.data, sel.ctypes.data, len(sel),
                                      _ptr(sums), cnt, _ptr(ws), wsb, _stream(sums.device)), "vge_stats_accumulate")
    counts[0], counts[1] = cnt[0], cnt[1]


def stats_finalize(sums: torch.Tensor, counts: np.ndarray, layout: str = "kp") -> Tuple[torch.Tensor, torch.Tensor]:
    """mean / std in the layout's feats column order (layout "nokp": [2356], the keypoint-less ModalityStats)."""
    lib = L.load()
    mean = torch.empty(FEAT_DIMS[layout], device=sums.device, dtype=torch.float32)
    std = torch.empty_like(mean)
    cnt = (C.c_int64 * 2)(int(counts[0]), int(counts[1]))
    L.check(lib.vge_stats_finalize_layout(_ptr(sums), cnt, LAYOUTS[layout], _ptr(mean), _ptr(std),
                                          _stream(sums.device)), "vge_stats_finalize")
    return mean, std


COMPUTE = {"f32": 0, "f32x3": 1, "f16": 2}


class Encoder:
    """HumanActionScorer (model.py:102-193) as a libvge encoder handle owning repacked HBM weights.

    compute="f32x3" (default): split-precision 3xfp16 MFMA, f32-class results (~1e-7 from exact f32);
    compute="f32": exact f32 MFMA.  n_modalities 5 (vit, global, pose, beta, kp2d; feats rows of 2596) or 4 (the
    keypoint-less model, feats rows of 2356).  A checkpoint with d_model / time_heads other than 256 / 8 runs on the
    generic exact-f32 kernels (compute "f32" only; d_model 32..256 in steps of 32, head dim <= 64): its embeddings
    are d_model wide."""

    def __init__(self, state_dict: Dict[str, np.ndarray], time_layers: int = 4, time_heads: int = 8,
                 d_model: int = 256, device=None, compute: str = "f32x3", n_modalities: int = 5):
        lib = L.load()
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        dims = L.Dims()
        dims.n_modalities = n_modalities
        for i in range(min(n_modalities, 5)):
            dims.dims_raw[i] = DIMS_RAW[i]
            dims.dims_diff[i] = DIMS_DIFF[i]
        dims.d_model, dims.time_layers, dims.time_heads, dims.clip_len = d_model, time_layers, time_heads, 32
        keep = []
        views = (L.TensorView * len(state_dict))()
        for i, (k, v) in enumerate(state_dict.items()):
            a = np.ascontiguousarray(np.asarray(v, np.float32))
            keep.append(a)
            views[i].name = k.encode()
            views[i].data = a.ctypes.data
            views[i].ndim = a.ndim
            for j, s in enumerate(a.shape[:4]):
                views[i].shape[j] = s
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            L.check(lib.vge_encoder_create(C.byref(dims), views, len(state_dict), COMPUTE[compute], C.byref(h)),
                    "vge_encoder_create")
        self.compute = compute
        self._h = h
        self._tail = None  # set_tail_stream()
        self._lib = lib
        self.capacity = 0
        self.n_modalities = n_modalities
        self.d_model = int(d_model)
        self.feat_dim = int(lib.vge_encoder_feat_dim(h))
        self.layout = "kp" if self.feat_dim == FEAT_DIM else "nokp"

    def reserve(self, max_windows: int) -> None:
        if max_windows > self.capacity:
            with torch.cuda.device(self.device):
                L.check(self._lib.vge_encoder_reserve(self._h, int(max_windows)), "vge_encoder_reserve")
            self.capacity = int(max_windows)

    def encode(self, feats: torch.Tensor, frame_embed: bool = False, tc: bool = True,
               seq_out: Optional[torch.Tensor] = None, tc_out: Optional[torch.Tensor] = None):
        """feats [B,32,feat_dim] -> (seq_embed [B,d], frame_embeds [B,33,d] | None, tc_window [B] | None), d = d_model.
        seq_out / tc_out: optional contiguous float32 destinations ([B,d] / [B]) written in place."""
        B, T, D = feats.shape
        if D != self.feat_dim:
            raise L.VgeError(f"feats last dim {D} != {self.feat_dim}")
        D_ = self.d_model
        for t, shape in ((seq_out, (B, D_)), (tc_out, (B,))):
            if t is not None and (tuple(t.shape) != shape or t.dtype != torch.float32 or not t.is_contiguous()
                                  or t.device != feats.device):
                raise L.VgeError(f"encode: output must be a contiguous float32 {shape} tensor on {feats.device}")
        self.reserve(B)
        seq = seq_out if seq_out is not None else torch.empty((B, D_), device=feats.device, dtype=torch.float32)
        fe = torch.empty((B, T + 1, D_), device=feats.device, dtype=torch.float32) if frame_embed else None
        tcw = (tc_out if tc_out is not None else torch.empty((B,), device=feats.device, dtype=torch.float32)) if tc else None
        L.check(self._lib.vge_encode(self._h, _ptr(feats), B, T, _ptr(seq), _ptr(fe), _ptr(tcw), _stream(feats.device)),
                "vge_encode")
        if self._tail is not None:
            # the outputs are written on the tail stream.  Those allocated here belong to the current stream in the
            # caching allocator's books: record the tail stream on them (a dropped fe / tcw is not reused before the
            # tail stream is done with it) and make the current stream wait for it, so they read as complete there.
            # Caller-provided seq_out / tc_out (and no frame embeddings) keep the overlap: the caller orders them.
            own = [t for t, given in ((seq, seq_out is not None), (fe, False), (tcw, tc_out is not None))
                   if t is not None and not given]
            for t in own:
                t.record_stream(self._tail)
            if own:
                torch.cuda.current_stream(feats.device).wait_stream(self._tail)
        return seq, fe, tcw

    def status(self) -> None:
        """Raise DeviceFaultError if a completed launch raised the encoder's device status word (vge_encoder_status;
        synchronise first to cover launches still in flight)."""
        L.check(self._lib.vge_encoder_status(self._h), "vge_encoder_status")

    def clear_status(self) -> None:
        L.check(self._lib.vge_encoder_clear_status(self._h), "vge_encoder_clear_status")

    def profile_mask(self, event_mask: int) -> None:
        """Stage-boundary events recorded by profiled encodes (bit k = before stage k; 0x3 = the conv stage only)."""
        L.check(self._lib.vge_encoder_profile_mask(self._h, event_mask), "vge_encoder_profile_mask")

    def wait_conv(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        """Make `stream` (default: the current stream) wait until the conv stage of the last encode() -- the last
        reader of its feats -- has finished (vge_encoder_wait_conv): the next batch can be featurised into the same
        buffer on another stream while this batch's fusion / transformer run."""
        st = (stream if stream is not None else torch.cuda.current_stream()).cuda_stream
        L.check(self._lib.vge_encoder_wait_conv(self._h, st), "vge_encoder_wait_conv")

    def set_tail_stream(self, stream: Optional[torch.cuda.Stream]) -> None:
        """Run the stages after the fusion (token GEMM, transformer, outputs / TC) of later encode() calls on `stream`
        (None: back on the encode stream) -- vge_encoder_set_tail_stream.  encode()'s outputs are then complete in
        `stream`'s order; the encode stream is free for the next batch's featurise and conv stage."""
        with torch.cuda.device(self.device):  # its events are created on the encoder's device
            L.check(self._lib.vge_encoder_set_tail_stream(self._h, stream.cuda_stream if stream is not None else None),
                    "vge_encoder_set_tail_stream")
        self._tail = stream

    STAGES = ("conv_encoders", "fusion_pool", "token_gemm", "transformer", "outputs_tc")

    def profile_begin(self, max_calls: int) -> None:
        L.check(self._lib.vge_encoder_profile_begin(self._h, int(max_calls)), "vge_encoder_profile_begin")

    def profile_read(self):
        """-> ({stage: summed ms}, n_calls) for the encode calls since profile_begin."""
        ms = (C.c_double * 5)()
        n = C.c_int(0)
        L.check(self._lib.vge_encoder_profile_read(self._h, ms, C.byref(n)), "vge_encoder_profile_read")
        return dict(zip(self.STAGES, list(ms))), int(n.value)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                self._lib.vge_encoder_destroy(h)
            except Exception:
                pass
            self._h = None


def tc_windows(frame_embeds: torch.Tensor) -> torch.Tensor:
    lib = L.load()
    B, T1, d = frame_embeds.shape
    out = torch.empty((B,), device=frame_embeds.device, dtype=torch.float32)
    L.check(lib.vge_tc_windows(_ptr(frame_embeds), B, T1, d, _ptr(out), _stream(frame_embeds.device)), "vge_tc_windows")
    return out


def score_videos(seq: torch.Tensor, tc_window: torch.Tensor, video_first_win: torch.Tensor, video_class: torch.Tensor,
                 centroids: Optional[torch.Tensor], out: Optional[Tuple[torch.Tensor, torch.Tensor]] = None
                 ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-video AC (float32) / TC (float64).  out: (ac [V] float32, tc [V] float64) to write instead of new device
    tensors -- device tensors, or pinned (page-locked) host tensors, which the kernel then writes directly over the
    bus (no copy kernels; the values are the host's once the stream is synchronised)."""
    lib = L.load()
    V = int(video_class.shape[0])
    d = int(seq.shape[1])
    if out is not None:
        ac, tc = out
        if (ac.dtype, tc.dtype) != (torch.float32, torch.float64) or ac.numel() < V or tc.numel() < V or \
                not ac.is_contiguous() or not tc.is_contiguous() or \
                any(not t.is_cuda and not t.is_pinned() for t in (ac, tc)):
            raise L.VgeError("score_videos: out must be contiguous (float32, float64) tensors of >= V elements, on the "
                             "device or in pinned host memory")
    else:
        ac = torch.empty((V,), device=seq.device, dtype=torch.float32)
        tc = torch.empty((V,), device=seq.device, dtype=torch.float64)
    if centroids is None:
        centroids = torch.zeros((1, d), device=seq.device, dtype=torch.float32)
    # (a pinned host tensor's address is also its device address: HIP maps page-locked host memory into the GPU's
    # virtual address space at the same address)
    op = lambda t: _ptr(t) if t.is_cuda else t.data_ptr()  # noqa: E731
    L.check(lib.vge_score_videos(_ptr(seq), _ptr(tc_window), _ptr(video_first_win), _ptr(video_class), _ptr(centroids),
                                 V, d, op(ac), op(tc), _stream(seq.device)), "vge_score_videos")
    return ac, tc


def centroid_accumulate(seq: torch.Tensor, class_id: torch.Tensor, sums: torch.Tensor, counts: torch.Tensor) -> None:
    lib = L.load()
    C_, d = sums.shape
    L.check(lib.vge_centroid_accumulate(_ptr(seq), _ptr(class_id), int(seq.shape[0]), C_, d, _ptr(sums), _ptr(counts),
                                        _stream(seq.device)), "vge_centroid_accumulate")


def centroid_finalize(sums: torch.Tensor, counts: torch.Tensor) -> torch.Tensor:
    lib = L.load()
    C_, d = sums.shape
    out = torch.empty_like(sums)
    L.check(lib.vge_centroid_finalize(_ptr(sums), _ptr(counts), C_, d, _ptr(out), _stream(sums.device)),
            "vge_centroid_finalize")
    return out
