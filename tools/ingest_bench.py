#!/usr/bin/env python3
"""Host ingest throughput: decode N synthetic 32-frame clips written in the
reference layout (np.savez_compressed npz + keypoints.npy) into a frame store three ways:

  numpy    -- np.load in a thread pool (the reference's reader; vge.eval.load_frame_store_numpy)
  native   -- libvge's zip/zlib decoder on native threads (vge.ingest.load_frame_store_native)
  sidecar  -- the packed uncompressed frame-store file (vge.ingest.load_sidecar)

and prints one JSON line of clips/s.  CPU only.

    python tools/ingest_bench.py [--clips 512] [--threads 16] [--dir /tmp/vge_ingest]
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "video-gen-evals_amd"))

from vge import ingest, synth  # noqa: E402
from vge.data import create_dataset_from_generated_meshes  # noqa: E402
from vge.eval import load_frame_store_numpy  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--clips", type=int, default=512)
ap.add_argument("--threads", type=int, default=min(16, os.cpu_count() or 1))
ap.add_argument("--dir", default=None)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()

work = Path(a.dir or tempfile.mkdtemp(prefix="vge_ingest_"))
gen, kps = work / "generated_meshes", work / "generated_kps"
if not gen.exists() or len(list(gen.glob("*.npz"))) < a.clips:
    for i in range(a.clips):
        name = synth.generated_name(i)
        c = synth.make_clip(synth.SEED_GEN, i, 32)
        synth.save_clip_npz(gen / f"{name}.npz", c)
        (kps / name).mkdir(parents=True, exist_ok=True)
        import numpy as np
        np.save(kps / name / "keypoints.npy", c.keypoints)
items = create_dataset_from_generated_meshes(str(gen)).items[: a.clips]
mb = sum(os.path.getsize(it.path) for it in items) / 1e6


def best(fn):
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    return min(ts), out


t_np, _ = best(lambda: load_frame_store_numpy(items, str(kps), True, workers=a.threads))
t_nat, st = best(lambda: ingest.load_frame_store_native(items, str(kps), True, threads=a.threads, pinned=False))
side = work / "store.vgefs"
ingest.save_sidecar(st, str(side))
t_side, _ = best(lambda: ingest.load_sidecar(str(side), pinned=False))
print(json.dumps({"clips": len(items), "threads": a.threads, "npz_MB": round(mb, 1),
                  "numpy_clips_per_s": round(len(items) / t_np, 1),
                  "native_clips_per_s": round(len(items) / t_nat, 1),
                  "sidecar_clips_per_s": round(len(items) / t_side, 1),
                  "native_speedup": round(t_np / t_nat, 2), "host_cpus": os.cpu_count()}))
if a.dir is None:
    shutil.rmtree(work, ignore_errors=True)
