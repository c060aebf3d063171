"""Summarise tools/prof_gemm.sh passes: per-dispatch averages of every counter for the kernels whose name contains
PATTERN (default gemm_bf16_kernel; Cijk for hipBLASLt's).   python tools/pmc_gemm_summary.py TAG [PATTERN]"""
import collections, csv, glob, json, sys
tag = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "gemm_bf16_kernel"
res = {}
for d in sorted(glob.glob(f"gpurun_out/pg_{tag}_*/")):
    for f in glob.glob(d + "*counter_collection.csv"):
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if pat not in r["Kernel_Name"]:
                continue
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in acc.items():
            res[k] = sum(v) / len(v) * (1 if True else 1)
    for f in glob.glob(d + "*kernel_stats.csv"):
        for r in csv.DictReader(open(f)):
            if pat in r["Name"]:
                res["avg_ns"] = float(r["AverageNs"])
print(json.dumps(res, indent=1))
