"""One 1x1 conv shape (YOLOX dark3 bottleneck 1x1: 64 x 80 x 80 x 128 -> 128) launched 5 times, for PMC passes."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "video-gen-evals_amd"))
import torch  # noqa: E402
from vge import dwpose as D  # noqa: E402
n, H, W, Cin, Cout = 64, 80, 80, int(sys.argv[1]) if len(sys.argv) > 1 else 128, 128
x = torch.randn(n, H, W, Cin, device="cuda").to(torch.bfloat16)
w = torch.randn(Cout, Cin, 1, 1, device="cuda") * 0.1
b = torch.zeros(Cout, device="cuda")
out = torch.empty(n, H, W, Cout, device="cuda", dtype=torch.bfloat16)
for _ in range(5):
    D.conv_bf16(x, w, b, out=out)
torch.cuda.synchronize()
