"""A/B timer of the conv-s2 GEMMs of one train step (bs 32, 256x256, bf16): the automatic plan (the halo kernel,
csrc/halo_bf16.hip, where it applies) against the automatic im2col plan (force {-2, 0}) and the 8-wave 256 x 128
halo block (force {HALO_CFG, 1}), interleaved rounds in
one process, HIP events over 20 launches each; prints us / TFLOP/s per shape and the relative output difference."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))

import torch  # noqa: E402

from stcgan_amd import _lib as L  # noqa: E402
from stcgan_amd import ops  # noqa: E402

BF = torch.bfloat16
SHAPES = [  # (kind, GEMM grid, cin, cout, what)
    (L.CONV_S2, 64, 64, 128, "e2 / D c2 fwd"),
    (L.CONV_S2, 32, 128, 256, "e3 / D c3 fwd"),
    (L.CONV_S2, 16, 256, 512, "e4 fwd (256 x 64 halo tile)"),
    (L.CONV_S2, 64, 64, 256, "d2 dgrad (ConvT 256->64)"),
    (L.CONV_S2, 32, 128, 512, "d3 dgrad (ConvT 512->128)"),
    (L.CONV_S2, 16, 256, 1024, "d4 dgrad (ConvT 1024->256)"),
    (L.CONVT_S2, 64, 256, 64, "d2 fwd (ConvT 256->64)"),
    (L.CONVT_S2, 32, 512, 128, "d3 fwd"),
    (L.CONVT_S2, 16, 1024, 256, "d4 fwd"),
    (L.CONVT_S2, 64, 128, 64, "e2 / D c2 dgrad"),
    (L.CONVT_S2, 32, 256, 128, "e3 / D c3 dgrad"),
    (L.CONVT_S2, 16, 512, 256, "e4 dgrad"),
    (L.CONV_S1, 31, 256, 512, "D c4 fwd (k4 s1)"),
    (L.CONV_S1_DGRAD, 32, 512, 256, "D c4 dgrad"),
]


def main():
    dev = torch.device("cuda", 0)
    B = 32
    g = torch.Generator(device=dev).manual_seed(0)
    for kind, gh, cin, cout, what in SHAPES:
        convt = kind == L.CONVT_S2
        ih, oh = {L.CONV_S2: (2 * gh, gh), L.CONVT_S2: (gh, 2 * gh), L.CONV_S1: (gh + 1, gh),
                  L.CONV_S1_DGRAD: (gh - 1, gh)}[kind]
        x = (torch.randn((B, ih, ih, cin), generator=g, device=dev)).to(BF)
        if convt:
            w = torch.randn((cin, cout, 4, 4), generator=g, device=dev) * 0.05
            wp = ops.pack(L.PACK_CONVT_FWD, w, cout, cin, BF)
        elif kind == L.CONV_S1_DGRAD:
            w = torch.randn((cin, cout, 4, 4), generator=g, device=dev) * 0.05
            wp = ops.pack(L.PACK_CONV_S1_DGRAD, w, cout, cin, BF)
        else:
            w = torch.randn((cout, cin, 4, 4), generator=g, device=dev) * 0.05
            wp = ops.pack(L.PACK_CONV_FWD, w, cout, cin, BF)
        ys = {}
        cands = (("halo", None), ("im2col", (-2, 0)), ("halo8w", (ops.HALO_CFG, 1)), ("n64w8", (ops.HALO_CFG, 4)))
        times = {c[0]: [] for c in cands}
        plans = {}
        for rnd in range(5):
            for name, force in cands:
                y = torch.empty((B, oh, oh, cout), device=dev, dtype=BF)
                plans[name] = ops.conv_query(kind, B, gh, gh, cin, cout, BF, force=force)[2]
                ops.conv_stats(kind, B, L.nhwc_view(x), cin, wp, cout, L.nhwc_view(y), BF, force=force)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    ops.conv_stats(kind, B, L.nhwc_view(x), cin, wp, cout, L.nhwc_view(y), BF, force=force)
                e1.record()
                e1.synchronize()
                times[name].append(e0.elapsed_time(e1) / 20 * 1e3)
                ys[name] = y
        fl = 2.0 * B * gh * gh * cout * 16 * cin
        d = float((ys["halo"].float() - ys["im2col"].float()).abs().max() / ys["im2col"].float().abs().max())
        line = f"{what:28s} grid{gh} cin{cin} cout{cout}:"
        for name, _ in cands:
            t = sorted(times[name])
            line += f"  {name} plan{list(plans[name])} med {t[2]:.1f} us min {t[0]:.1f} ({fl / t[0] / 1e6:.0f} TF)"
        print(line + f"  rel diff {d:.2e}", flush=True)


if __name__ == "__main__":
    main()
