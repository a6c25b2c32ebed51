"""Loader-wave GEMM tiles (igemm_bf16 configs 29-32: 4 waves that only issue LDS-DMA beside the compute
waves) against the automatic plan on the step's large conv problems: output bit-identity against the
same-size plain tile, then HIP-graph-replayed times (scripts/tune_bf16.bench)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import torch  # noqa: E402

import tune_bf16  # noqa: E402
from stcgan_amd import _lib as L  # noqa: E402
from stcgan_amd import ops  # noqa: E402

B = 32
PROBS = [  # (name, prob, plain cfg of the same tile for the bit-identity check, loader cfgs)
    ("e2 conv_s2 64x64 64->128", (L.CONV_S2, B, 64, 64, 128, 128, 64, 64, 64, 128), 0, (33, 29, 31)),
    ("e3 conv_s2 32x32 128->256", (L.CONV_S2, B, 32, 32, 64, 64, 32, 32, 128, 256), 0, (33, 29, 31)),
    ("d4 convT 16x16 1024->256", (L.CONVT_S2, B, 16, 16, 16, 16, 32, 32, 1024, 256), 0, (33, 29, 31)),
    ("d3 convT 32x32 512->128", (L.CONVT_S2, B, 32, 32, 32, 32, 64, 64, 512, 128), 0, (33, 29, 31)),
    ("d2 convT 64x64 256->64", (L.CONVT_S2, B, 64, 64, 64, 64, 128, 128, 256, 64), 11, (34, 32)),
    ("e4 conv_s2 16x16 256->512", (L.CONV_S2, B, 16, 16, 32, 32, 16, 16, 256, 512), 0, (33, 29, 31)),
]


def run_once(prob, force):
    kind, b, gh, gw, xh, xw, yh, yw, cin, cout = prob
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(7)
    x = (torch.randn((b, xh, xw, cin), device=dev, generator=g) * 0.5).to(torch.bfloat16)
    taps, nph = (4, 4) if kind == L.CONVT_S2 else (16, 1)
    w = (torch.randn((nph, cout, taps, cin), device=dev, generator=g) * 0.05).to(torch.bfloat16)
    y = torch.zeros((b, yh, yw, cout), device=dev, dtype=torch.bfloat16)
    part, nch = ops.conv_stats(kind, b, L.nhwc_view(x), cin, w, cout, L.nhwc_view(y), torch.bfloat16, force=force)
    torch.cuda.synchronize()
    return y, part


def main():
    for name, prob, plain, lds in PROBS:
        kind, b, gh, gw, xh, xw, yh, yw, cin, cout = prob
        taps, nph = (4, 4) if kind == L.CONVT_S2 else (16, 1)
        fl = 2.0 * b * gh * gw * nph * cout * taps * cin
        y0, p0 = run_once(prob, (plain, 1))
        t_auto = tune_bf16.bench(prob, None, reps=20)
        line = f"{name:28s} auto {t_auto:7.1f} us {fl / t_auto / 1e6:6.0f} TF"
        for c in lds:
            y1, p1 = run_once(prob, (c, 1))
            same = torch.equal(y0.view(torch.int16), y1.view(torch.int16))
            t = tune_bf16.bench(prob, (c, 1), reps=20)
            line += f" | cfg{c} {t:7.1f} us {fl / t / 1e6:6.0f} TF {'bit-identical' if same else 'DIFFERS'}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
