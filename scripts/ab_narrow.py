"""The full-resolution narrow ConvT layers at bs=32 (G output layer 128x128x128 -> 256x256x{1,3} fp32 NCHW + tanh;
first-layer input gradient 128x128x64 -> 256x256x8 bf16 NHWC): the streaming kernel (default) against the tiled
K-split kernel (force {4, 1}), HIP events over 20 calls, HBM rate on the compulsory bytes (input once, output once)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402

from stcgan_amd import _lib as L, ops  # noqa: E402

BF = torch.bfloat16
dev = "cuda"


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


B, G = 32, 128
for cin, n, f32 in ((128, 1, True), (128, 3, True), (64, 8, False)):
    x = torch.randn((B, G, G, cin), device=dev).to(BF)
    w = torch.randn((cin, n, 4, 4), device=dev) * 0.05
    wp = ops.pack(L.PACK_CONVT_FWD, w, n, cin, BF)
    b = torch.randn(n, device=dev)
    if f32:
        y = torch.empty((B, n, 2 * G, 2 * G), device=dev)
        yv = L.nchw_view(y)
    else:
        y = torch.empty((B, 2 * G, 2 * G, n), device=dev, dtype=BF)
        yv = L.nhwc_view(y)
    byt = B * G * G * cin * 2 + y.numel() * y.element_size()
    res = []
    forces = [None, (4, 1)] + ([(4, 32), (6, 32)] if cin == 128 else [(6, 32)])
    for force in forces:
        t = timed(lambda: ops.conv(L.CONVT_S2, B, L.nhwc_view(x), cin, wp, n, yv, BF, bias=b if f32 else None,
                                   tanh=f32, out_f32=f32, force=force))
        res.append(t)
    print(f"ConvT {cin}->{n} ({'fp32 NCHW + tanh' if f32 else 'bf16 NHWC'}): stream {res[0]:6.1f} us "
          f"({byt / res[0] / 1e6:.2f} TB/s)  tiled {res[1]:6.1f} us ({byt / res[1] / 1e6:.2f} TB/s)  " +
          "  ".join(f"stream NS={f[0]} {t:6.1f} us" for f, t in zip(forces[2:], res[2:])), flush=True)
