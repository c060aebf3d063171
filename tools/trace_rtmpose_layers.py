"""One RTMPose-l call (256 whole-frame instances) twice, for a rocprofv3 --kernel-trace per-layer breakdown."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "video-gen-evals_amd"))
import torch  # noqa: E402
from vge import dwpose as D, synth  # noqa: E402
ex = D.DwposeExtractor(synth.make_rtmpose_state_dict(D.RTMPOSE_L), D.RTMPOSE_L, device="cuda:0", max_instances=256)
frames = torch.from_numpy(synth.make_frames(3, 256)).cuda()
for _ in range(2):
    ex.keypoints(frames)
    torch.cuda.synchronize()
