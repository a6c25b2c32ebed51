"""GPU time (graph-replayed, no host overhead) of the deep-layer conv + split-K reduce/stats under forced
split-K; tile config 5 (64x64)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402

from stcgan_amd import _lib as L  # noqa: E402
from stcgan_amd import ops  # noqa: E402

BF = torch.bfloat16
dev = torch.device("cuda", 0)
CASES = [(L.CONV_S2, 32, 8, 8, 512, 512), (L.CONV_S2, 32, 4, 4, 512, 512), (L.CONV_S2, 32, 2, 2, 512, 512),
         (L.CONV_S2, 32, 1, 1, 512, 512), (L.CONVT_S2, 32, 1, 1, 512, 512), (L.CONVT_S2, 32, 2, 2, 1024, 512),
         (L.CONVT_S2, 32, 4, 4, 1024, 512)]
for kind, B, gh, gw, cin, cout in CASES:
    if kind == L.CONVT_S2:
        xh, xw, yh, yw, nph, taps = gh, gw, 2 * gh, 2 * gw, 4, 4
    else:
        xh, xw, yh, yw, nph, taps = 2 * gh, 2 * gw, gh, gw, 1, 16
    x = (torch.randn((B, xh, xw, cin), device=dev) * 0.5).to(BF)
    y = torch.empty((B, yh, yw, cout), device=dev, dtype=BF)
    w = (torch.randn((nph, cout, taps, cin), device=dev) * 0.05).to(BF)
    res = []
    for ks in (0, 2, 4, 8, 16, 32, 64):
        force = None if ks == 0 else (5, ks)
        try:
            ops.conv_stats(kind, B, L.nhwc_view(x), cin, w, cout, L.nhwc_view(y), BF, force=force)
        except Exception as e:  # noqa: BLE001
            res.append(f"ks{ks}:err")
            continue
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            for _ in range(2):
                ops.conv_stats(kind, B, L.nhwc_view(x), cin, w, cout, L.nhwc_view(y), BF, force=force)
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                for _ in range(20):
                    ops.conv_stats(kind, B, L.nhwc_view(x), cin, w, cout, L.nhwc_view(y), BF, force=force)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            g.replay()
        e1.record()
        e1.synchronize()
        res.append(f"ks{ks}:{e0.elapsed_time(e1) / 100 * 1e3:5.1f}")
    print(f"kind {kind} grid {gh}x{gw} cin {cin} cout {cout}: " + "  ".join(res))
