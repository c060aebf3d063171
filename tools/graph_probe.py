"""Config-2 step (featurise -> encode -> per-video scores into pinned host memory, 256 clips) eager vs replayed from a
HIP graph captured once (torch.cuda.graph over the libvge launches), interleaved rounds on one box.
python tools/graph_probe.py [rounds] [steps] -> JSON"""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "video-gen-evals_amd"))
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from vge import ops, synth  # noqa: E402
from vge.data import pack_frame_store  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 100
dev = torch.device("cuda", 0)
V = 256
clips = bench.make_clips(synth.SEED_GEN, 0, V, 32)
store = ops.DeviceFrameStore.from_host(pack_frame_store(clips, [f"g{i}" for i in range(V)], ["X"] * V), dev)
rng = np.random.default_rng(0)
mean = torch.from_numpy(rng.normal(0, 0.1, ops.FEAT_DIM).astype(np.float32)).to(dev)
std = torch.from_numpy(rng.uniform(0.5, 2.0, ops.FEAT_DIM).astype(np.float32)).to(dev)
enc = ops.Encoder(synth.make_state_dict(synth.DIMS_RAW, synth.DIMS_DIFF), device=dev, compute="f32x3")
enc.reserve(V)
win = torch.tensor([[v, 0] for v in range(V)], dtype=torch.int32, device=dev)
first = torch.arange(0, V + 1, dtype=torch.int32, device=dev)
vcls = torch.tensor([v % 10 for v in range(V)], dtype=torch.int32, device=dev)
cent = torch.nn.functional.normalize(torch.randn(10, 256), dim=-1).to(dev)
feats = torch.empty((V, 32, ops.FEAT_DIM), device=dev)
seq = torch.empty((V, 256), device=dev)
tcw = torch.empty((V,), device=dev)
hac = torch.empty((V,), dtype=torch.float32, pin_memory=True)
htc = torch.empty((V,), dtype=torch.float64, pin_memory=True)


def step():
    ops.featurize(store, win, mean, std, out=feats)
    enc.encode(feats, frame_embed=False, tc=True, seq_out=seq, tc_out=tcw)
    ops.score_videos(seq, tcw, first, vcls, cent, out=(hac, htc))


enc.profile_mask(0)
s = torch.cuda.Stream(device=dev)
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        step()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
ref = (hac.clone(), htc.clone())
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    step()
torch.cuda.synchronize()
hac.zero_()
g.replay()
torch.cuda.synchronize()
same = bool(torch.equal(hac, ref[0]) and torch.equal(htc, ref[1]))


def timed(fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / steps * 1e3


res = {"eager_ms": [], "graph_ms": [], "graph_equals_eager": same, "steps": steps}
for _ in range(rounds):
    res["eager_ms"].append(timed(step))
    res["graph_ms"].append(timed(g.replay))
print(json.dumps(res))
