"""First-layer conv (B=32, 256^2 x 8 -> 128^2 x 64, LeakyReLU epilogue): the row-halo kernel vs the GEMM tile,
HIP events around 50 back-to-back calls each (STC_HALO8, STC_HALO8_GRID = persistent blocks per CU)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402

from stcgan_amd import _lib as L  # noqa: E402
from stcgan_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
B = 32
x = torch.randn((B, 256, 256, 8), device=dev).to(torch.bfloat16)
w = (torch.randn((1, 64, 16, 8), device=dev) * 0.1).to(torch.bfloat16)
y = torch.empty((B, 128, 128, 64), device=dev, dtype=torch.bfloat16)
mb = (x.numel() + y.numel()) * 2 / 1e6


def run(halo, grid=None, reps=50):
    os.environ["STC_HALO8"] = "1" if halo else "0"
    if grid:
        os.environ["STC_HALO8_GRID"] = str(grid)
    for _ in range(3):
        ops.conv_act(L.CONV_S2, B, L.nhwc_view(x), 8, w, 64, L.nhwc_view(y), 0.2, torch.bfloat16)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        ops.conv_act(L.CONV_S2, B, L.nhwc_view(x), 8, w, 64, L.nhwc_view(y), 0.2, torch.bfloat16)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for _ in range(2):
    t0 = run(False)
    line = f"gemm tile {t0:6.1f} us ({mb / t0:.2f} TB/s compulsory)"
    for g in (1, 2, 4, 8):
        t = run(True, g)
        line += f" | halo {g}/CU {t:6.1f} us ({mb / t:.2f} TB/s)"
    print(line, flush=True)
