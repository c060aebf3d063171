#!/usr/bin/env python3
"""Standalone featurise timing (vge_featurize on the bench's 256 clips, 50 back-to-back launches, hipEvents) for a
given libvge.so (env VGE_LIB); with the VGE_ABL featurise ablation builds (1024: vit part only, 2048: without it) it
splits the kernel's time between its parts.  Usage: VGE_LIB=... python tools/time_featurize.py TAG
"""
import sys, json, torch
sys.path.insert(0, "video-gen-evals_amd"); sys.path.insert(0, ".")
import bench
from vge import ops, synth
from vge.data import pack_frame_store
dev = torch.device("cuda", 0)
clips = bench.make_clips(synth.SEED_GEN, 0, 256, 32)
st = ops.DeviceFrameStore.from_host(pack_frame_store(clips, [f"g{i}" for i in range(256)], ["X"] * 256), dev)
win = torch.tensor([[v, 0] for v in range(256)], dtype=torch.int32, device=dev)
mean = torch.zeros(ops.FEAT_DIM, device=dev); std = torch.ones(ops.FEAT_DIM, device=dev)
out = torch.empty((256, 32, ops.FEAT_DIM), device=dev)
for _ in range(5): ops.featurize(st, win, mean, std, out=out)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50): ops.featurize(st, win, mean, std, out=out)
e1.record(); torch.cuda.synchronize()
print(sys.argv[1], round(e0.elapsed_time(e1) / 50, 4), "ms")
