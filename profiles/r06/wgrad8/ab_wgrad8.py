"""A/B of the 8-wide halo weight-gradient tile (cfg 8) against the im2col loader tile (cfg 7, round 5's plan) on the
train step's P = 2048 weight gradients (bs 32, 8 x 8 D grids), HIP events, interleaved rounds."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "shadow-removal-istd_amd"))
import torch
from stcgan_amd import _lib as L, ops
BF = torch.bfloat16
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
SH = [("e5 conv 16->8: D = dy 8x8x512, G = x 16x16x512", 8, 512, 16, 512),
      ("d5 ConvT 8->16: D = x 8x8x1024, G = dy 16x16x512", 8, 1024, 16, 512)]
for what, gd, R, gg, Cg in SH:
    D = torch.randn((32, gd, gd, R), generator=g, device=dev).to(BF)
    G = torch.randn((32, gg, gg, Cg), generator=g, device=dev).to(BF)
    res = {}
    for rnd in range(5):
        for name, force in (("im2col cfg7", (7, 0)), ("halo cfg8", (8, 0)), ("auto", None)):
            dW = ops.wgrad(32, 2, L.nhwc_view(D), R, L.nhwc_view(G), Cg, Cg, BF, device=dev, force=force)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                dW = ops.wgrad(32, 2, L.nhwc_view(D), R, L.nhwc_view(G), Cg, Cg, BF, device=dev, force=force)
            e1.record(); e1.synchronize()
            t, ref = res.get(name, ([], None))
            t.append(e0.elapsed_time(e1) / 20 * 1e3)
            res[name] = (t, dW.clone())
    fl = 2.0 * 32 * gd * gd * R * 16 * Cg
    base = res["im2col cfg7"][1]
    for name, (t, dW) in res.items():
        t = sorted(t)
        err = float((dW - base).abs().max() / base.abs().max())
        print(f"{what}: {name:12s} med {t[2]:6.1f} us min {t[0]:6.1f} ({fl / t[0] / 1e6:5.0f} TF)  rel diff vs cfg7 {err:.1e}",
              flush=True)
