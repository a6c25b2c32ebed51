"""Fused BatchNorm-backward input gradients (stc_conv_bwd_bn + stc_bn_bwd_apply, as the train step calls them) at
bs 32 against the plain conv of the same shape: what the BN-backward epilogue costs.  HIP events over 20 calls."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402

from stcgan_amd import _lib as L, ops  # noqa: E402

BF = torch.bfloat16
dev = torch.device("cuda", 0)
B = 32
CASES = [  # kind, Cin, Cout, GH (GEMM grid), C, ch_off, what
    (L.CONV_S2, 64, 256, 64, 128, 128, "d2 dgrad"), (L.CONV_S2, 128, 512, 32, 256, 256, "d3 dgrad"),
    (L.CONV_S2, 256, 1024, 16, 512, 512, "d4 dgrad"), (L.CONVT_S2, 256, 128, 32, 128, 0, "e3 dgrad"),
    (L.CONVT_S2, 128, 64, 64, 64, 0, "e2 dgrad")]


def timed(fn):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / 20 * 1e3


for kind, cin, cout, gh, C, off, what in CASES:
    ih, oh = (2 * gh, gh) if kind == L.CONV_S2 else (gh, 2 * gh)
    dy = torch.randn((B, ih, ih, cin), device=dev).to(BF)
    if kind == L.CONV_S2:
        w = ops.pack(L.PACK_CONV_FWD, torch.randn((cout, cin, 4, 4), device=dev) * 0.05, cout, cin, BF)
    else:
        w = ops.pack(L.PACK_CONVT_FWD, torch.randn((cin, cout, 4, 4), device=dev) * 0.05, cout, cin, BF)
    out = torch.empty((B, oh, oh, cout), device=dev, dtype=BF)
    x = torch.randn((B, oh, oh, C), device=dev).to(BF)
    go = torch.randn((B, oh, oh, C), device=dev).to(BF) if off == C else None
    dx = torch.empty((B, oh, oh, C), device=dev, dtype=BF)
    st = tuple(torch.rand(C, device=dev) + 0.5 for _ in range(4))
    gam = torch.rand(C, device=dev) + 0.5
    tb, tc = [], []
    for _ in range(5):
        tb.append(timed(lambda: ops.conv_bn_backward(kind, B, L.nhwc_view(dy), cin, w, cout, L.nhwc_view(out), BF,
                                                     bn_x=L.nhwc_view(x), C=C, bn_state=st, gamma=gam, s_self=0.2,
                                                     ch_off=off, g_other=L.nhwc_view(go) if go is not None else None,
                                                     s_other=0.0, dxv=L.nhwc_view(dx))))
        tc.append(timed(lambda: ops.conv(kind, B, L.nhwc_view(dy), cin, w, cout, L.nhwc_view(out), BF)))
    print(f"{what:9s}: conv + BN-backward sums + apply {sorted(tb)[2]:6.1f} us   plain conv {sorted(tc)[2]:6.1f} us",
          flush=True)
