"""Per-layer kernel times of the gate detector from a rocprofv3 kernel-trace database (tools/time_frcnn.py under
`rocprofv3 --kernel-trace`): the last detect chunk's dispatches, labelled in vge_frcnn.cpp's launch order.
Usage: python tools/frcnn_layers.py <run_results.db | run_kernel_trace.csv> [depth] -> per-layer table + per-kind totals."""
import sqlite3
import sys
from collections import defaultdict


def labels(depth=101, stem_fused=True):
    """stem_fused: the stem conv + max pool as one dispatch (frcnn_stem_pool_kernel, the default since round 6)"""
    nb = {50: (3, 4, 6, 3), 101: (3, 4, 23, 3), 152: (3, 8, 36, 3)}[depth]
    L = ["resize_h", "resize_v"] + (["stem_pool"] if stem_fused else ["stem", "maxpool"])
    for s, n in enumerate(nb):
        for b in range(n):
            p = f"res{s + 2}.{b}"
            if b == 0:
                L.append(p + ".shortcut")
            L += [p + ".conv1", p + ".conv2(g)", p + ".conv3"]
    L += ["fpn_lat5", "fpn_out5"]
    for l in (4, 3, 2):
        L += [f"upsample{l}", f"fpn_lat{l}", f"fpn_out{l}"]
    L.append("p6")
    for l in range(2, 7):
        L += [f"rpn_conv_p{l}", f"rpn_head_p{l}"]
    L += ["rpn_select", "rpn_nms", "rpn_merge", "roi_align", "fc1", "fc2", "predictor", "det_post"]
    return L


def main():
    db = sys.argv[1]
    depth = int(sys.argv[2]) if len(sys.argv) > 2 else 101
    if db.endswith(".csv"):  # rocprofv3 --output-format csv: run_kernel_trace.csv
        import csv
        rs = sorted(csv.DictReader(open(db)), key=lambda r: int(r["Start_Timestamp"]))
        rows = [(r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), int(r["Grid_Size_X"]),
                 int(r["Workgroup_Size_X"])) for r in rs]
    else:
        c = sqlite3.connect(db)
        rows = c.execute("select name, duration, grid_x, workgroup_x from kernels order by start").fetchall()
    rows = [r for r in rows if not r[0].startswith("__amd_rocclr") and "at::" not in r[0]]
    lab = labels(depth, any("frcnn_stem_pool" in r[0] for r in rows))
    last = rows[-len(lab):]
    if not last[-1][0].startswith("_ZN12_GLOBAL__N_115det_post") and "det_post" not in last[-1][0]:
        print("warning: the trace does not end with det_post_kernel")
    kind = defaultdict(float)
    tot = 0.0
    for l, (name, dur, gx, wx) in zip(lab, last):
        short = name.split("(")[0][-60:]
        k = l.split(".")[-1] if l.startswith("res") else l.rstrip("0123456789").rstrip("_p")
        kind[k] += dur / 1e3
        tot += dur / 1e3
        print(f"{l:24s} {dur / 1e3:9.1f} us  grid {gx // max(wx, 1):7d}  {short}")
    print(f"total {tot:.1f} us per chunk")
    for k, v in sorted(kind.items(), key=lambda kv: -kv[1]):
        print(f"  {k:18s} {v:9.1f} us  {100 * v / tot:5.1f} %")


if __name__ == "__main__":
    main()
