"""Dump the gate detector's outputs on a fixed frame pool (for bitwise A/B of libvge.so builds: VGE_LIB selects one).
python tools/frcnn_dump.py OUT.pt [frames] [chunk] -> torch.save({dets, n_dets, person, n_person})"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "video-gen-evals_amd"))
from vge import synth  # noqa: E402
from vge.frcnn import FRCNN_X101, FrcnnDetector  # noqa: E402

out = sys.argv[1]
nf = int(sys.argv[2]) if len(sys.argv) > 2 else 64
chunk = int(sys.argv[3]) if len(sys.argv) > 3 else 64
det = FrcnnDetector(synth.make_gate_frcnn_state_dict(FRCNN_X101), FRCNN_X101, device="cuda", chunk=chunk)
fr = torch.from_numpy(synth.make_frame_pool(9400, nf)).cuda()
taps = det.make_taps(nf, 256, 256)
o = det.detect(fr, taps=taps)
torch.cuda.synchronize()
torch.save({**{k: v.cpu() for k, v in o.items()}, "fpn": [t.cpu() for t in taps["fpn"]]}, out)
print("dumped", out, int(o["n_dets"].sum()))
