"""HBM rate of the BN element-wise passes on the train step's big shapes (bf16 NHWC, B=32):
bn_apply (1 read + 1-2 writes) and bn_backward without statistics (3 reads + 1 write), HIP events."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402

from stcgan_amd import _lib as L, ops  # noqa: E402

dev = "cuda"
dt = torch.bfloat16
B = 32


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for H, C in ((128, 64), (64, 128), (32, 256), (16, 512)):
    x = torch.randn(B, H, H, C, device=dev).to(dt)
    y1 = torch.empty_like(x)
    y2 = torch.empty_like(x)
    sc = torch.rand(C, device=dev) + 0.5
    sh = torch.randn(C, device=dev)
    n = x.numel() * 2
    us = timed(lambda: ops.bn_apply(B, L.nhwc_view(x), C, dt, (sc, sh), L.nhwc_view(y1), 0.2))
    us2 = timed(lambda: ops.bn_apply(B, L.nhwc_view(x), C, dt, (sc, sh), L.nhwc_view(y1), 0.2, L.nhwc_view(y2), 0.0))
    g1 = torch.randn_like(x)
    g2 = torch.randn_like(x)
    us3 = timed(lambda: ops.bn_backward(B, L.nhwc_view(x), C, dt, L.nhwc_view(y1), g1=L.nhwc_view(g1), s1=0.2,
                                        g2=L.nhwc_view(g2), s2=0.0))
    print(f"{H}x{H}x{C}: apply {us:6.1f} us {2 * n / us / 1e3:5.2f} GB/s | apply2 {us2:6.1f} us "
          f"{3 * n / us2 / 1e3:5.2f} GB/s | bwd(no stats) {us3:6.1f} us {4 * n / us3 / 1e3:5.2f} GB/s", flush=True)
