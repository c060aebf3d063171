#!/usr/bin/env python3
"""HBM traffic (FETCH_SIZE x 2 + WRITE_SIZE, the MI355X_MICROARCH.md HBM recipe) and L2 hit rate per launch of the
step's other kernels from the PMC passes of tools/profile_round.sh TAG (last 6 dispatches of each kernel = the timed
steps), written to profiles/pmc_kernels.json (bench.py's stage_roofline reads it while each kernel's sources are
unchanged: `source_sha`).   python tools/pmc_kernels.py TAG [WINDOWS_PER_LAUNCH]"""
import collections
import csv
import glob
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402  (KERNEL_SOURCES / sources_sha: the hash bench.py checks)
tag = sys.argv[1]
windows = int(sys.argv[2]) if len(sys.argv) > 2 else 256
KERNELS = {"transformer_x3_kernel": "fused transformer (model.py:145-146,187-193)",
           "featurize_tiles_kernel": "featurise (utils.py:383-516)", "fuse_kernel": "fusion pool (model.py:79-98)",
           "conv_encoder_f16w_kernel": "conv encoders, f16 unit kernel", "score_videos_kernel": "AC/TC per video"}


def counters(kind, pat):
    per = collections.defaultdict(dict)
    for f in glob.glob(str(ROOT / "gpurun_out" / f"prof_{tag}_{kind}" / "**" / "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                d = per[int(r["Dispatch_Id"])]
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    keep = [per[k] for k in sorted(per)[-6:]]
    out = collections.defaultdict(float)
    for d in keep:
        for k, v in d.items():
            out[k] += v / len(keep)
    return dict(out), len(keep)


res = {}
for pat, what in KERNELS.items():
    f, n = counters("fetch", pat)
    w, _ = counters("write", pat)
    l2, _ = counters("l2", pat)
    if not n:
        continue
    hit = l2.get("TCC_HIT_sum", 0.0)
    res[pat] = {"what": what, "dispatches": n, "hbm_bytes_per_launch": (f.get("FETCH_SIZE", 0) * 2 + w.get("WRITE_SIZE", 0)) * 1024,
                "windows_per_launch": windows, "l2_hit_rate": hit / max(1.0, hit + l2.get("TCC_MISS_sum", 0.0)),
                "source_sha": bench.sources_sha(bench.KERNEL_SOURCES[pat]) if pat in bench.KERNEL_SOURCES else None,
                "source": f"gpurun_out/prof_{tag}_*/ (tools/profile_round.sh {tag})"}
(ROOT / "profiles" / "pmc_kernels.json").write_text(json.dumps(res, indent=1) + "\n")
print(json.dumps(res, indent=1))
