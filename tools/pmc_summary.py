#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection CSVs per kernel (mean over dispatches).
    python tools/pmc_summary.py DIR [DIR ...] [--kernel substr]"""
import collections
import csv
import glob
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
ksub = None
if "--kernel" in sys.argv:
    ksub = sys.argv[sys.argv.index("--kernel") + 1]
    args = [a for a in args if a != ksub]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for d in args:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if ksub and ksub not in k:
                continue
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, d in agg.items():
    print(k[:90])
    print("   dispatch_ns(mean) %.0f" % (sum(dur[k]) / len(dur[k])))
    for c, v in sorted(d.items()):
        print("   %-32s %.4g  (n=%d)" % (c, sum(v) / len(v), len(v)))
