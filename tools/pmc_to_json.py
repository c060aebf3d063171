#!/usr/bin/env python3
"""Condense the rocprofv3 passes of tools/profile_round.sh into profiles/pmc_conv_encoder.json (read by
bench.py for roofline.traffic) and a per-kernel stats CSV under profiles/.

    python tools/pmc_to_json.py TAG COMPUTE [--windows 256]

Only the timed-workload dispatches are kept: the last --last conv-encoder dispatches of the run (bench.py
--steps in tools/profile_round.sh; setup launches come first).  HBM bytes = FETCH_SIZE x 2 (gfx950 reports half of wide streaming reads,
MI355X_MICROARCH.md HBM section) + WRITE_SIZE, both in KB as rocprofv3 reports them.
"""
import argparse
import collections
import csv
import glob
import json
import shutil
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
import sys  # noqa: E402
sys.path.insert(0, str(ROOT))
ap = argparse.ArgumentParser()
ap.add_argument("tag")
ap.add_argument("compute")
ap.add_argument("--windows", type=int, default=256)
ap.add_argument("--last", type=int, default=6)
a = ap.parse_args()
out_dir = ROOT / "gpurun_out"
KNAME = {"f32x3": "conv_encoder_x3s_kernel",
         "f16": "conv_encoder_x3s_kernel" if __import__("bench").f16_conv_is_x3s() else "conv_encoder_f16w_kernel",
         "f32": "conv_encoder_kernel("}[a.compute]


def rows(kind):
    for f in glob.glob(str(out_dir / f"prof_{a.tag}_{kind}" / "**" / "*counter_collection.csv"), recursive=True):
        yield from csv.DictReader(open(f))


def counters(kind):
    per_dispatch = collections.defaultdict(dict)
    for r in rows(kind):
        if KNAME in r["Kernel_Name"]:
            d = per_dispatch[int(r["Dispatch_Id"])]
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    keep = [per_dispatch[k] for k in sorted(per_dispatch)[-a.last:]]
    vals = collections.defaultdict(list)
    for d in keep:
        for k, v in d.items():
            vals[k].append(v)
    return {k: sum(v) / len(v) for k, v in vals.items()}, len(keep)


fetch, nf = counters("fetch")
write, nw = counters("write")
l2, _ = counters("l2")
sq, _ = counters("sq")
# kernel-trace average of the same dispatches
tr = []
for f in glob.glob(str(out_dir / f"prof_{a.tag}_trace" / "**" / "*kernel_trace.csv"), recursive=True):
    rs = [r for r in csv.DictReader(open(f)) if KNAME in r["Kernel_Name"]]
    rs.sort(key=lambda r: int(r["Dispatch_Id"]))
    tr += [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs[-a.last:]]
hbm = fetch["FETCH_SIZE"] * 1024 * 2 + write["WRITE_SIZE"] * 1024
res = {
    "kernel": KNAME.rstrip("("), "source_sha": __import__("bench")._kernel_sources_sha(), "windows_per_launch": a.windows, "dispatches": {"fetch": nf, "write": nw},
    "fetch_size_kb_raw": fetch["FETCH_SIZE"], "write_size_kb": write["WRITE_SIZE"],
    "hbm_bytes_per_launch": hbm, "hbm_bytes_per_window": hbm / a.windows,
    "l2_hit_rate": l2["TCC_HIT_sum"] / (l2["TCC_HIT_sum"] + l2["TCC_MISS_sum"]) if l2 else None,
    "kernel_trace_avg_ms": sum(tr) / len(tr) / 1e6 if tr else None,
    "sq": sq, "source": f"gpurun_out/prof_{a.tag}_*/ (tools/profile_round.sh {a.tag} {a.compute})",
}
if sq.get("GRBM_GUI_ACTIVE") and tr:
    res["clock_ghz_est"] = sq["GRBM_GUI_ACTIVE"] / 8 / (sum(tr) / len(tr))   # GRBM counts summed over 8 XCDs
pj = ROOT / "profiles" / "pmc_conv_encoder.json"
allj = json.loads(pj.read_text()) if pj.exists() else {}
allj[a.compute] = res
pj.write_text(json.dumps(allj, indent=1) + "\n")
for f in glob.glob(str(out_dir / f"prof_{a.tag}_trace" / "**" / "*kernel_stats.csv"), recursive=True):
    shutil.copy(f, ROOT / "profiles" / f"rocprof_{a.tag}_kernel_stats.csv")
print(json.dumps(res, indent=1))
