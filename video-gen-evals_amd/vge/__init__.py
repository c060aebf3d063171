"""vge — MI355X-native Action-Consistency / Temporal-Coherence scoring (XThomasBU/video-gen-evals).

Host code mirroring the reference's eval.py / utils.py interfaces over ``libvge.so``, a C-ABI
library of hand-written gfx950 HIP kernels (featurisation, the fusion encoder on f32 MFMA,
centroid accumulation and the AC/TC reductions).  There is no CPU fallback: the compute entry
points raise if the library cannot be loaded.
"""
__all__ = ["data", "synth"]
