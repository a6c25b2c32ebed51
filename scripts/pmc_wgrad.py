"""Run one bf16 weight-gradient problem (auto plan) N times: the program for per-kernel PMC passes.
usage: pmc_wgrad.py B s dh dw gh gw R Cg reps"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402

from stcgan_amd import _lib as L  # noqa: E402

B, s, dh, dw, gh, gw, R, Cg, reps = map(int, sys.argv[1:10])
dev = torch.device("cuda", 0)
d = (torch.randn((B, dh, dw, R), device=dev) * 0.5).to(torch.bfloat16)
g = (torch.randn((B, gh, gw, Cg), device=dev) * 0.5).to(torch.bfloat16)
dv, gv = L.nhwc_view(d), L.nhwc_view(g)
lib = L.lib()
ws_b = ctypes.c_int64()
assert lib.stc_conv_wgrad_query(L.BF16, B, dh, dw, R, Cg, None, ctypes.byref(ws_b), None) == 0
ws = torch.empty(max(int(ws_b.value), 16), dtype=torch.uint8, device=dev)
dW = torch.empty((R, Cg, 4, 4), device=dev)


def call():
    rc = lib.stc_conv_wgrad_ex(L.BF16, B, s, dv, R, None, None, 0, 0.0, gv, Cg, Cg, None, None, 0, 0.0, L.ptr(dW), None,
                               L.ptr(ws), int(ws_b.value), L.stream())
    assert rc == 0, lib.stc_last_error().decode()


for _ in range(3):
    call()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    call()
e1.record()
e1.synchronize()
t = e0.elapsed_time(e1) / reps
fl = 2.0 * B * dh * dw * R * 16 * Cg
print(f"{t * 1e3:.1f} us/call (kernel + reduce, incl. host gaps), {fl / (t * 1e-3) / 1e12:.1f} TF")
