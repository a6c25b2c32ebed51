"""The PatchGAN logits layer's weight gradient at bs=32 (x 31x31x512 bf16, dy 30x30x8 with 1 real channel):
stc_conv_wgrad_rows (MFMA kernel + ordered reduce) per call, HIP events over 20 calls; HBM rate on x once."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402

from stcgan_amd import _lib as L, ops  # noqa: E402

BF = torch.bfloat16
dev = "cuda"
B, C = 32, 512
x = torch.randn((B, 31, 31, C), device=dev).to(BF)
dy = torch.zeros((B, 30, 30, 8), device=dev).to(BF)
dy[..., 0] = torch.randn((B, 30, 30), device=dev).to(BF)


def call():
    return ops.wgrad(B, 1, L.nhwc_view(dy), 8, L.nhwc_view(x), C, C, BF, device=dev, rows=1, rows_kernel=True)


call()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    call()
e1.record()
e1.synchronize()
us = e0.elapsed_time(e1) / 20 * 1e3
print(f"logits wgrad (rows, bs=32): {us:.1f} us per call ({x.numel() * 2 / us / 1e6:.2f} TB/s on x)", flush=True)
