"""Host cost of the pieces one launch is made of (us per call): ctypes call overhead, view building, torch.empty,
event fork, and one small library launch (bn_apply on a tiny tensor) end to end."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402

from stcgan_amd import _lib as L, ops  # noqa: E402


def per_call(fn, n=20000):
    fn()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t) / n * 1e6


lib = L.lib()
dev = torch.device("cuda", 0)
x = torch.randn(2, 4, 4, 64, device=dev).to(torch.bfloat16)
y = torch.empty_like(x)
sc = torch.rand(64, device=dev)
sh = torch.rand(64, device=dev)
v = L.nhwc_view(x)
s = L.stream()
print(f"ctypes stc_version()            {per_call(lambda: lib.stc_version()):6.2f} us")
print(f"L.stream()                      {per_call(L.stream):6.2f} us")
print(f"L.nhwc_view(t)                  {per_call(lambda: L.nhwc_view(x)):6.2f} us")
print(f"L.ptr(t)                        {per_call(lambda: L.ptr(sc)):6.2f} us")
print(f"torch.empty NHWC bf16           {per_call(lambda: torch.empty((32, 64, 64, 128), dtype=torch.bfloat16, device=dev)):6.2f} us")
f = lib.stc_bn_apply
yv = L.nhwc_view(y)
ps, ph = L.ptr(sc), L.ptr(sh)
print(f"stc_bn_apply raw ctypes launch  {per_call(lambda: f(1, 2, v, 64, ps, ph, yv, 0.2, L.NULL_VIEW, 0.0, s)):6.2f} us")
print(f"ops.bn_apply (wrapper)          {per_call(lambda: ops.bn_apply(2, L.nhwc_view(x), 64, torch.bfloat16, (sc, sh), L.nhwc_view(y), 0.2)):6.2f} us")
torch.cuda.synchronize()
side = torch.cuda.Stream()
cur = torch.cuda.current_stream()
ev = torch.cuda.Event()


def fork():
    ev.record(cur)
    side.wait_event(ev)


print(f"event fork (record + wait)      {per_call(fork):6.2f} us")
print(f"tensor.fill_(0) (ATen launch)   {per_call(lambda: sc.fill_(0)):6.2f} us")
torch.cuda.synchronize()
