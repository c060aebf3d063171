#!/usr/bin/env python3
"""Per-layer time and TFLOP/s of YOLOX-L from a rocprofv3 --kernel-trace of tools/yolox_prof.py: the conv dispatches of
the last detect chunk, paired in order with the layer list of vge_yolox.cpp's forward (CSP = conv1|conv2 fused, then
Bottleneck 1x1 + 3x3 per block, then conv3; head cls0|reg0 fused).   python tools/yolox_layers.py gpurun_out/DIR [n]"""
import csv
import glob
import sys

d, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 64
S, w0, dep, hc = 640, 64, 3, 256
L = []


def cv(name, hw, cin, cout, k, stride=1):
    L.append((name, 2.0 * n * hw * hw * cin * cout * k * k, f"{k}x{k} {cin}->{cout} @{hw}"))


def csp(name, hw, cin, cout, nb):
    hid = cout // 2
    cv(name + ".c12", hw, cin, 2 * hid, 1)
    for b in range(nb):
        cv(f"{name}.m{b}.1x1", hw, hid, hid, 1)
        cv(f"{name}.m{b}.3x3", hw, hid, hid, 3)
    cv(name + ".c3", hw, 2 * hid, cout, 1)


h2, h4, h8, h16, h32 = S // 2, S // 4, S // 8, S // 16, S // 32
c3, c4, c5 = 4 * w0, 8 * w0, 16 * w0
cv("stem", h2, 16, w0, 3); cv("d2", h4, w0, 2 * w0, 3); csp("c2", h4, 2 * w0, 2 * w0, dep)
cv("d3", h8, 2 * w0, c3, 3); csp("c3", h8, c3, c3, 3 * dep); cv("d4", h16, c3, c4, 3); csp("c4", h16, c4, c4, 3 * dep)
cv("d5", h32, c4, c5, 3); cv("spp1", h32, c5, c5 // 2, 1); cv("spp2", h32, 2 * c5, c5, 1); csp("c5", h32, c5, c5, dep)
cv("lat0", h32, c5, c4, 1); csp("p4", h16, 2 * c4, c4, dep); cv("red1", h16, c4, c3, 1); csp("p3", h8, 2 * c3, c3, dep)
cv("bu2", h16, c3, c3, 3); csp("n3", h16, 2 * c3, c4, dep); cv("bu1", h32, c4, c4, 3); csp("n4", h32, 2 * c4, c5, dep)
for g, cin in ((h8, c3), (h16, c4), (h32, c5)):
    cv(f"head{g}.stem", g, cin, hc, 1); cv(f"head{g}.first", g, hc, 2 * hc, 3); cv(f"head{g}.cls1", g, hc, hc, 3)
    cv(f"head{g}.reg1", g, hc, hc, 3); cv(f"head{g}.regobj", g, hc, 8, 1); cv(f"head{g}.cls0", g, hc, 1, 1)
rows = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
starts = [i for i, r in enumerate(rows) if "letterbox_focus" in r[2]]
chunk = [r for r in rows[starts[-1]:] if ("conv" in r[2] and "bf16" in r[2]) or "Cijk_" in r[2]]  # library GEMMs too
assert len(chunk) == len(L), (len(chunk), len(L))
tot_ms = tot_fl = 0.0
agg = {}
for (nm, fl, desc), (t0, t1, kn) in zip(L, chunk):
    ms = (t1 - t0) / 1e6
    tot_ms += ms
    tot_fl += fl
    key = desc
    a = agg.setdefault(key, [0, 0.0, 0.0, kn.split("(")[0].replace("void (anonymous namespace)::", "")])
    a[0] += 1; a[1] += ms; a[2] += fl
for key, (cnt, ms, fl, kn) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{ms:7.3f} ms {100 * ms / tot_ms:5.1f}%  {fl / ms / 1e9:6.0f} TF/s  x{cnt:<2d} {key:24s} {kn}")
print(f"chunk: {tot_ms:.2f} ms, {tot_fl / 1e12:.2f} TFLOP, {tot_fl / tot_ms / 1e9:.0f} TF/s")
