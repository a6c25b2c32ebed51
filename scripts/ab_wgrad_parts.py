"""The train step's weight-gradient problems one at a time (5 calls each), for a rocprofv3 kernel trace that separates
the main tile from the ordered split reduce: which share of each call the reduce is."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402

from stcgan_amd import _lib as L, ops  # noqa: E402

BF = torch.bfloat16
dev = "cuda"
B = 32
SHAPES = [  # stride, D grid (H = W), R, Cg (the forward conv: G grid = 2 x D grid)
    (2, 64, 128, 64), (2, 32, 256, 128), (2, 32, 512, 128), (2, 16, 512, 256), (2, 16, 1024, 256),
    (2, 64, 256, 64), (2, 128, 64, 8), (2, 128, 128, 8), (2, 8, 1024, 512), (2, 4, 1024, 512), (2, 1, 512, 512),
    (1, 31, 512, 256)]
for stride, gd, R, Cg in SHAPES:
    gg = gd + 1 if stride == 1 else 2 * gd
    D = torch.randn((B, gd, gd, R), device=dev).to(BF)
    G = torch.randn((B, gg, gg, Cg), device=dev).to(BF)
    ws, plan = ops.wgrad_query(B, gd, gd, R, Cg, BF)
    for _ in range(5):
        ops.wgrad(B, stride, L.nhwc_view(D), R, L.nhwc_view(G), Cg, Cg, BF, device=dev)
    torch.cuda.synchronize()
    print(f"stride {stride} D {gd}x{gd}x{R} G {gg}x{gg}x{Cg}: plan {plan}", flush=True)
