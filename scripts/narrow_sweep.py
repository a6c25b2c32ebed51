"""Time the narrow-N kernels under forced tile shapes {rows, 16-column blocks (+16: the row-split
narrow_halo_kernel instead of the K-split narrow_wk_kernel)} (stc_conv_fwd_ex hook)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402

from stcgan_amd import _lib as L  # noqa: E402
from stcgan_amd._lib import lib, ptr, stream, check  # noqa: E402

dev = torch.device("cuda", 0)
BF = torch.bfloat16
CASES = [  # name, kind, B, grid H, W, cin, cout, out (nchw fp32 + tanh | nhwc bf16)
    ("G out convT 128->1", L.CONVT_S2, 32, 128, 128, 128, 1, "nchw"),
    ("G out convT 128->3", L.CONVT_S2, 32, 128, 128, 128, 3, "nchw"),
    ("e1 dgrad convT 64->8", L.CONVT_S2, 32, 128, 128, 64, 8, "nhwc"),
    ("D logits s1 512->1", L.CONV_S1, 32, 30, 30, 512, 1, "nhwc1"),
]
SHAPES = [None, (8, 17), (8, 18), (16, 17), (8, 1), (8, 2), (16, 1), (4, 1), (4, 2)]
ws = torch.empty(256 << 20, dtype=torch.uint8, device=dev)
for name, kind, B, gh, gw, cin, cout, out in CASES:
    if kind == L.CONVT_S2:
        xh, xw, yh, yw, nph, taps = gh, gw, 2 * gh, 2 * gw, 4, 4
    else:
        xh, xw, yh, yw, nph, taps = gh + 1, gw + 1, gh, gw, 1, 16
    x = (torch.randn((B, xh, xw, cin), device=dev) * 0.5).to(BF)
    npad = 8
    w = (torch.randn((nph, npad, taps, cin), device=dev) * 0.05).to(BF)
    bias = torch.randn(cout, device=dev)
    if out == "nchw":
        y = torch.empty((B, cout, yh, yw), device=dev)
        yv, tanh, f32 = L.nchw_view(y), 1, 1
    else:
        y = torch.empty((B, yh, yw, npad), device=dev, dtype=BF)
        yv, tanh, f32 = L.nhwc_view(y), 0, 0
    ref = None
    for sh in SHAPES:
        fp = (ctypes.c_int32 * 2)(*sh) if sh else None
        def call():  # noqa: E306
            check(lib().stc_conv_fwd_ex(L.dtype_code(BF), kind, B, L.nhwc_view(x), cin, ptr(w), cout if out != "nhwc" else npad,
                                        yv, ptr(bias) if out != "nhwc" else None, tanh, f32, None, 0, fp, ptr(ws),
                                        ws.numel(), stream()), "stc_conv_fwd_ex")
        try:
            call()
        except RuntimeError as e:
            print(f"{name:22s} {str(sh):8s} -- {e}")
            continue
        torch.cuda.synchronize()
        if ref is None:
            ref = y.clone()
        err = float((y.float() - ref.float()).abs().max())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            call()
        e1.record()
        e1.synchronize()
        t = e0.elapsed_time(e1) / 20 * 1e3
        mb = (x.numel() * 2 + y.numel() * y.element_size()) / 1e6
        print(f"{name:22s} {str(sh):8s} {t:7.1f} us  {mb / t:5.2f} TB/s  maxdiff {err:.2e}")
