"""Per-layer algorithmic bytes / FLOPs of the gate detector (X101-32x8d-FPN) next to the measured time and PMC bytes.

Inputs: a `tools/profile_e2e.sh TAG` run's frcnn passes (gpurun_out/pe_TAG_frcnn_{trace,fetch,write}/: the kernel
trace of tools/time_frcnn.py and its FETCH_SIZE / WRITE_SIZE passes).  The last detect call's dispatches are labelled
in vge_frcnn.cpp's launch order (tools/frcnn_layers.py).  Per layer and per frame:

  alg_MB   the bytes the layer must move once: its input activation + its output (+ the residual / the FPN top-down
           input it adds) in the kernels' own formats (NHWC bf16, the stem's 8-channel padded input, f32 RPN outputs),
           + its weights once per chunk
  pmc_MB   FETCH_SIZE x 2 + WRITE_SIZE (MI355X_MICROARCH.md: FETCH_SIZE counts half of a 16-B-per-lane streaming read;
           other access widths are uncalibrated, so a ratio far from 1 on a gather kernel may be the counter, not bytes)
  GF       algorithmic GFLOP (grouped convs at their grouped size)
  us       the trace pass's duration of the dispatch, per chunk; TB/s and TF/s from alg_MB and GF over it

Usage: python tools/frcnn_layer_bytes.py TAG [frames_per_chunk] [H W] [-o] -> table on stdout (+ profiles/frcnn_layer_bytes_TAG.json with -o)."""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
from frcnn_layers import labels  # noqa: E402


def layer_shapes(H=800, W=800, depth=101):
    """label -> (alg bytes per frame, weight bytes per chunk, flop per frame) for the 800 x 800 padded input."""
    nb = {50: (3, 4, 6, 3), 101: (3, 4, 23, 3), 152: (3, 8, 36, 3)}[depth]
    B = 2  # bf16
    L = {}
    px = lambda h, w: h * w  # noqa: E731
    L["resize_h"] = (256 * 256 * 3 + 256 * W * 3, 0, 0)
    L["resize_v"] = (256 * W * 3 + H * W * 8 * B, 0, 0)
    h, w = H // 2, W // 2
    L["stem"] = (H * W * 8 * B + px(h, w) * 64 * B, 64 * 7 * 7 * 8 * B, 2.0 * px(h, w) * 64 * 3 * 49)
    L["maxpool"] = (px(h, w) * 64 * B + px(h // 2, w // 2) * 64 * B, 0, 0)
    L["stem_pool"] = (H * W * 8 * B + px(h // 2, w // 2) * 64 * B, L["stem"][1], L["stem"][2])  # fused: no stem output
    h, w = h // 2, w // 2
    cin, width, cout = 64, 256, 256
    lv = {}
    for s, n in enumerate(nb):
        for b in range(n):
            p = f"res{s + 2}.{b}"
            st = 2 if (b == 0 and s > 0) else 1
            ho, wo = (h - 1) // st + 1, (w - 1) // st + 1
            ci = cin if b == 0 else cout
            if b == 0:
                L[p + ".shortcut"] = (px(h, w) * ci * B + px(ho, wo) * cout * B, ci * cout * B,
                                      2.0 * px(ho, wo) * cout * ci)
            L[p + ".conv1"] = (px(h, w) * (ci + width) * B, ci * width * B, 2.0 * px(h, w) * width * ci)
            L[p + ".conv2(g)"] = (px(h, w) * width * B + px(ho, wo) * width * B, width * (width // 32) * 9 * B,
                                  2.0 * px(ho, wo) * width * (width // 32) * 9)
            L[p + ".conv3"] = (px(ho, wo) * (width + 2 * cout) * B, width * cout * B, 2.0 * px(ho, wo) * cout * width)
            h, w = ho, wo
        lv[s] = (h, w, cout)
        cin, width, cout = cout, width * 2, cout * 2
    F = 256
    h5, w5, c5 = lv[3]
    L["fpn_lat5"] = (px(h5, w5) * (c5 + F) * B, c5 * F * B, 2.0 * px(h5, w5) * F * c5)
    L["fpn_out5"] = (px(h5, w5) * 2 * F * B, F * F * 9 * B, 2.0 * px(h5, w5) * F * F * 9)
    for l in (4, 3, 2):
        hl, wl, cl = lv[l - 2]
        hu, wu, _ = lv[l - 1]
        L[f"upsample{l}"] = (px(hu, wu) * F * B + px(hl, wl) * F * B, 0, 0)
        L[f"fpn_lat{l}"] = (px(hl, wl) * (cl + 2 * F) * B, cl * F * B, 2.0 * px(hl, wl) * F * cl)
        L[f"fpn_out{l}"] = (px(hl, wl) * 2 * F * B, F * F * 9 * B, 2.0 * px(hl, wl) * F * F * 9)
    h6, w6 = (h5 - 1) // 2 + 1, (w5 - 1) // 2 + 1
    L["p6"] = (px(h5, w5) * F * B + px(h6, w6) * F * B, 0, 0)
    sizes = [lv[0][:2], lv[1][:2], lv[2][:2], lv[3][:2], (h6, w6)]
    for i, (hl, wl) in enumerate(sizes):
        L[f"rpn_conv_p{i + 2}"] = (px(hl, wl) * 2 * F * B, F * F * 9 * B, 2.0 * px(hl, wl) * F * F * 9)
        L[f"rpn_head_p{i + 2}"] = (px(hl, wl) * (F * B + 16 * 4), 15 * F * B, 2.0 * px(hl, wl) * 15 * F)
    P, fc = 1000, 1024
    L["rpn_select"] = (sum(px(a, b) * 16 * 4 for a, b in sizes), 0, 0)
    L["rpn_nms"] = (5 * 1024 * 8 * 4 * 2, 0, 0)
    L["rpn_merge"] = (5 * 1024 * 8 * 4 + P * 5 * 4, 0, 0)
    # output + every P2..P5 feature it samples read once (the lower bound: the 4 corners x 4 samples of a bin overlap)
    L["roi_align"] = (P * 49 * F * B + sum(px(a, b) for a, b in sizes[:4]) * F * B, 0, 0)
    L["fc1"] = (P * 49 * F * B + P * fc * B, fc * 49 * F * B, 2.0 * P * fc * 49 * F)
    L["fc2"] = (P * fc * 2 * B, fc * fc * B, 2.0 * P * fc * fc)
    L["predictor"] = (P * fc * B + P * 408 * 4, 401 * fc * B, 2.0 * P * 401 * fc)
    L["det_post"] = (P * 408 * 4 + P * 5 * 4, 0, 0)
    return L


def per_dispatch(path, counter):
    out = {}
    for f in Path(path).glob("**/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                d = int(r["Dispatch_Id"])
                nm, v = out.get(d, (r["Kernel_Name"], 0.0))
                out[d] = (nm, v + float(r["Counter_Value"]) * 1024)
    return out


def last_call(rows, lab):
    """the last len(lab) product dispatches, ending in det_post"""
    rows = [r for r in rows if not r[1].startswith("__amd_rocclr") and "at::" not in r[1]]
    last = rows[-len(lab):]
    assert "det_post" in last[-1][1], "the trace does not end with det_post_kernel"
    return last


def main():
    pos = [a for a in sys.argv[1:] if a != "-o"]
    tag = pos[0]
    chunk = int(pos[1]) if len(pos) > 1 else 64
    H = int(pos[2]) if len(pos) > 2 else 800
    W = int(pos[3]) if len(pos) > 3 else 800
    OUT = ROOT / "gpurun_out"
    tr = list(csv.DictReader(open(next((OUT / f"pe_{tag}_frcnn_trace").glob("**/*kernel_trace.csv")))))
    lab = labels(101, any("frcnn_stem_pool" in r["Kernel_Name"] for r in tr))
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    trows = last_call([(0, r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
                       for r in tr], lab)
    fe = per_dispatch(OUT / f"pe_{tag}_frcnn_fetch", "FETCH_SIZE")
    wr = per_dispatch(OUT / f"pe_{tag}_frcnn_write", "WRITE_SIZE")
    frows = last_call([(d, nm, v) for d, (nm, v) in sorted(fe.items())], lab)
    wrows = last_call([(d, nm, v) for d, (nm, v) in sorted(wr.items())], lab)
    shapes = layer_shapes(H, W)
    res, kind = [], defaultdict(lambda: defaultdict(float))
    print(f"{'layer':18s} {'us':>8s} {'alg_MB':>8s} {'pmc_MB':>8s} {'pmc/alg':>7s} {'TB/s':>6s} {'GF':>7s} {'TF/s':>6s}")
    for l, t, f, w in zip(lab, trows, frows, wrows):
        ab, wb, fl = shapes[l]
        alg = ab + wb / chunk
        pmc = (2 * f[2] + w[2]) / chunk
        us = t[2]
        k = l.split(".")[-1] if l.startswith("res") else l.rstrip("0123456789").rstrip("_p")
        stage = l.split(".")[0] if l.startswith("res") else k
        kname = t[1][t[1].find("::") + 2:] if "namespace)::" in t[1] else t[1]
        res.append({"layer": l, "kernel": kname.split("(")[0][:60], "us_per_chunk": us, "alg_bytes_per_frame": alg,
                    "pmc_bytes_per_frame": pmc, "gflop_per_frame": fl / 1e9})
        for key in (f"kind:{k}", f"stage:{stage}", "total"):
            kind[key]["us"] += us
            kind[key]["alg"] += alg
            kind[key]["pmc"] += pmc
            kind[key]["gf"] += fl / 1e9
        tbs = alg * chunk / (us * 1e-6) / 1e12 if us else 0
        tfs = fl * chunk / (us * 1e-6) / 1e12 if us else 0
        print(f"{l:18s} {us:8.1f} {alg / 1e6:8.2f} {pmc / 1e6:8.2f} {pmc / max(alg, 1):7.2f} {tbs:6.2f} "
              f"{fl / 1e9:7.2f} {tfs:6.0f}")
    print()
    summ = {}
    for key in sorted(kind, key=lambda k: -kind[k]["us"]):
        v = kind[key]
        summ[key] = {"us_per_chunk": v["us"], "alg_MB_per_frame": v["alg"] / 1e6, "pmc_MB_per_frame": v["pmc"] / 1e6,
                     "gflop_per_frame": v["gf"], "pmc_over_alg": v["pmc"] / max(v["alg"], 1)}
        print(f"{key:22s} {v['us']:9.1f} us  alg {v['alg'] / 1e6:8.1f} MB  pmc {v['pmc'] / 1e6:8.1f} MB  "
              f"x{v['pmc'] / max(v['alg'], 1):5.2f}  {v['gf']:7.1f} GF")
    if "-o" in sys.argv:
        dst = ROOT / "profiles" / f"frcnn_layer_bytes_{tag}.json"
        dst.write_text(json.dumps({"tag": tag, "chunk": chunk, "frame_hw_padded": [H, W], "layers": res,
                                   "summary": summ}, indent=1) + "\n")
        print("->", dst)


if __name__ == "__main__":
    main()
