"""Timing experiment: per-tile GEMM TFLOP/s of one G1+G2 forward with and without the
fused BN/activation load prologue (the no-prologue numbers are numerically wrong)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
from stcgan_amd import networks, ops  # noqa: E402

dt = sys.argv[1] if len(sys.argv) > 1 else "bf16"
B = 32
g1 = networks.get_generator(3, 1, ngf=64).cuda().set_compute_dtype(dt)
g2 = networks.get_generator(4, 3, ngf=64).cuda().set_compute_dtype(dt)
g1.apply(networks.weights_init)
g2.apply(networks.weights_init)
x = torch.rand(B, 3, 256, 256, device="cuda") * 2 - 1
for mode in [False, True, False, True]:
    ops._DEBUG_NO_PROLOGUE = mode
    with torch.no_grad():
        for _ in range(2):
            g2([x, g1(x)])
        torch.cuda.synchronize()
        ops._timer = []
        g2([x, g1(x)])
        torch.cuda.synchronize()
        launches, ops._timer = ops._timer, None
    per = {}
    for name, fl, e0, e1 in launches:
        a = per.setdefault(name, [0.0, 0.0])
        a[0] += fl
        a[1] += e0.elapsed_time(e1)
    tot = sum(v[1] for v in per.values())
    print(f"{dt} no_prologue={mode}: conv total {tot:.3f} ms; " +
          ", ".join(f"{k} {v[0] / v[1] / 1e9:.0f}TF/{v[1]:.3f}ms" for k, v in sorted(per.items(), key=lambda kv: -kv[1][1])[:5]))
