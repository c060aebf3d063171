import sys, torch
sys.path.insert(0, '/root/repo/video-gen-evals_amd')
from vge import dwpose as D, synth
det = D.YoloxDetector(synth.make_yolox_state_dict(D.YOLOX_L), D.YOLOX_L, device="cuda:0", chunk=64)
frames = torch.from_numpy(synth.make_frames(3, 64)).cuda()
det.detect(frames); torch.cuda.synchronize()
det.detect(frames); torch.cuda.synchronize()
