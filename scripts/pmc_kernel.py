"""Run one bf16 conv problem (forced tile plan) N times: the program for per-kernel PMC passes.
usage: pmc_kernel.py kind B gh gw cin cout cfg ks reps"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402

from stcgan_amd import _lib as L  # noqa: E402
from stcgan_amd import ops  # noqa: E402

kind, B, gh, gw, cin, cout, cfg, ks, reps = map(int, sys.argv[1:10])
BF = torch.bfloat16
dev = torch.device("cuda", 0)
if kind == L.CONVT_S2:
    xh, xw, yh, yw = gh, gw, 2 * gh, 2 * gw
elif kind == L.CONV_S2:
    xh, xw, yh, yw = 2 * gh, 2 * gw, gh, gw
else:
    xh, xw, yh, yw = gh + 1, gw + 1, gh, gw
x = (torch.randn((B, xh, xw, cin), device=dev) * 0.5).to(BF)
y = torch.empty((B, yh, yw, cout), device=dev, dtype=BF)
taps = 4 if kind == L.CONVT_S2 else 16
nph = 4 if kind == L.CONVT_S2 else 1
w = (torch.randn((nph, cout, taps, cin), device=dev) * 0.05).to(BF)
force = None if cfg < 0 else (cfg, ks)
for _ in range(reps):
    ops.conv_stats(kind, B, L.nhwc_view(x), cin, w, cout, L.nhwc_view(y), BF, force=force)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    ops.conv_stats(kind, B, L.nhwc_view(x), cin, w, cout, L.nhwc_view(y), BF, force=force)
e1.record()
e1.synchronize()
t = e0.elapsed_time(e1) / reps
fl = 2.0 * B * gh * gw * nph * cout * taps * cin
print(f"{t * 1e3:.1f} us/launch (incl. host gaps), {fl / (t * 1e-3) / 1e12:.1f} TF")
