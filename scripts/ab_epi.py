"""Epilogue cost of the halo conv kernels: the same launch with the fused BatchNorm statistics (stc_conv_fwd_ex,
conv_stats) and without (stc_conv_fwd), bs 32 bf16, HIP events over 20 launches, interleaved rounds."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402

from stcgan_amd import _lib as L, ops  # noqa: E402

BF = torch.bfloat16
dev = torch.device("cuda", 0)
B = 32
SHAPES = [(L.CONV_S2, 64, 64, 128, "e2 fwd"), (L.CONV_S2, 32, 128, 256, "e3 fwd"), (L.CONVT_S2, 32, 512, 128, "d3 fwd"),
          (L.CONV_S1, 31, 256, 512, "D c4 fwd")]


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


for kind, gh, cin, cout, what in SHAPES:
    ih, oh = {L.CONV_S2: (2 * gh, gh), L.CONVT_S2: (gh, 2 * gh), L.CONV_S1: (gh + 1, gh)}[kind]
    x = torch.randn((B, ih, ih, cin), device=dev).to(BF)
    if kind == L.CONVT_S2:
        wp = ops.pack(L.PACK_CONVT_FWD, torch.randn((cin, cout, 4, 4), device=dev) * 0.05, cout, cin, BF)
    else:
        wp = ops.pack(L.PACK_CONV_FWD, torch.randn((cout, cin, 4, 4), device=dev) * 0.05, cout, cin, BF)
    y = torch.empty((B, oh, oh, cout), device=dev, dtype=BF)
    ts, tn = [], []
    for _ in range(5):
        ts.append(timed(lambda: ops.conv_stats(kind, B, L.nhwc_view(x), cin, wp, cout, L.nhwc_view(y), BF)))
        tn.append(timed(lambda: ops.conv(kind, B, L.nhwc_view(x), cin, wp, cout, L.nhwc_view(y), BF)))
    print(f"{what:10s}: with BN statistics {sorted(ts)[2]:6.1f} us   without {sorted(tn)[2]:6.1f} us   plan "
          f"{ops.conv_query(kind, B, gh, gh, cin, cout, BF)[2]}", flush=True)
