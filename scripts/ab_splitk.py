"""A/B timer of the deep levels' split-K GEMMs (bs 32, 256x256 generator, bf16): conv + BatchNorm statistics +
finalize per launch, for forced (tile config, splits) plans, split-K combined in the launch (each tile's last
arriver) or by the separate reduction kernel.  HIP events over 20 repetitions, interleaved rounds, median.

  python scripts/ab_splitk.py
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))

import torch  # noqa: E402

from stcgan_amd import _lib as L  # noqa: E402
from stcgan_amd import ops  # noqa: E402

BF = torch.bfloat16
B = 32
SHAPES = [  # (kind, GEMM grid, cin, cout, level)
    (L.CONV_S2, 8, 512, 512, "e5"), (L.CONV_S2, 4, 512, 512, "e6"), (L.CONV_S2, 2, 512, 512, "e7"),
    (L.CONVT_S2, 1, 512, 512, "d8"), (L.CONVT_S2, 2, 1024, 512, "d7"), (L.CONVT_S2, 4, 1024, 512, "d6"),
]
PLANS = [None, (12, 2), (12, 4), (12, 8), (5, 4), (5, 8), (5, 16)]


def main():
    dev = torch.device("cuda", 0)
    bn = torch.nn.BatchNorm2d(512).to(dev)
    t = torch.empty((2, 512), device=dev)
    for kind, g, cin, cout, what in SHAPES:
        if kind == L.CONVT_S2:
            x = torch.randn((B, g, g, cin), device=dev).to(BF)
            y = torch.empty((B, 2 * g, 2 * g, cout), device=dev, dtype=BF)
            w = (torch.randn((4, cout, 4, cin), device=dev) * 0.05).to(BF)
        else:
            x = torch.randn((B, 2 * g, 2 * g, cin), device=dev).to(BF)
            y = torch.empty((B, g, g, cout), device=dev, dtype=BF)
            w = (torch.randn((1, cout, 16, cin), device=dev) * 0.05).to(BF)
        runs = {}
        for plan in PLANS:
            for il in (True, False):
                ops.set_splitk_inlaunch(il)
                try:
                    _, _, po = ops.conv_query(kind, B, g, g, cin, cout, BF, force=plan)
                except RuntimeError:
                    continue
                runs[(plan, il)] = (po, [])

        def once(plan, il):
            ops.set_splitk_inlaunch(il)
            part, nch = ops.conv_stats(kind, B, L.nhwc_view(x), cin, w, cout, L.nhwc_view(y), BF, force=plan)
            ops.bn_finalize_part(part, nch, cout, bn, t[0], t[1])

        for key in runs:
            once(*key)
        torch.cuda.synchronize()
        for _ in range(5):
            for key, (po, ts) in runs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    once(*key)
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) / 20 * 1e3)
        for (plan, il), (po, ts) in sorted(runs.items(), key=lambda kv: statistics.median(kv[1][1])):
            print(f"{what} {'auto' if plan is None else plan} plan {list(po[:3])} "
                  f"{'in-launch' if il else 'reduce  '} {statistics.median(ts):7.1f} us", flush=True)
    ops.set_splitk_inlaunch(True)


if __name__ == "__main__":
    main()
