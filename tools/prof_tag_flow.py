import sys, time, cProfile, pstats
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/video-gen-evals_amd')
import bench_tag
from vge.dist import run_eval_distributed
p = bench_tag._dataset(0, 1)
f = lambda: run_eval_distributed(p["gen"], p["real"], p["ckpt"], p["gen_kp"], p["real_kp"], out_json=None, device="cuda:0")
f()
pr = cProfile.Profile(); pr.enable(); f(); pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
