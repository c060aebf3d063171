#!/usr/bin/env python3
"""Per-(kernel, grid) totals of a rocprofv3 --kernel-trace run: which launches of a multi-layer network take the time.
    python tools/kernel_trace_summary.py gpurun_out/DIR [--top 30]"""
import argparse
import collections
import csv
import glob

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--top", type=int, default=30)
a = ap.parse_args()
tot = collections.defaultdict(lambda: [0, 0.0])
for f in glob.glob(f"{a.dir}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"][:70]
        grid = (r.get("Grid_Size_X") or r.get("Grid_Size") or "?", r.get("Workgroup_Size_X") or "?",
                r.get("LDS_Block_Size") or r.get("Lds_Size") or "?")
        k = (name, grid)
        tot[k][0] += 1
        tot[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
all_ms = sum(v[1] for v in tot.values())
for (name, grid), (n, ms) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:a.top]:
    print(f"{ms:9.3f} ms {100 * ms / all_ms:5.1f}%  x{n:<4d} grid {grid[0]:>8} wg {grid[1]:>4} lds {grid[2]:>6}  {name}")
print(f"total {all_ms:.3f} ms")
