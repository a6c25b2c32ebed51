"""Loader-wave weight-gradient tiles (wgrad_bf16 configs 6/7: 4 waves that only issue LDS-DMA beside the 4
compute waves, 4- / 3-stage ring) against the automatic plan on the step's 128x128-tile problems: result
bit-identity against the plain tile at the same pixel splits, then HIP-graph-replayed times (kernel + split
reduction, scripts/tune_wgrad.bench)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import torch  # noqa: E402

import tune_wgrad  # noqa: E402
from stcgan_amd import _lib as L  # noqa: E402

PROBS = [  # (B, s, dh, dw, gh, gw, R, Cg, Cg_out)
    ("wg s2 P=131072 R128 Cg64", (32, 2, 64, 64, 128, 128, 128, 64, 64)),
    ("wg s2 P=32768 R256 Cg128", (32, 2, 32, 32, 64, 64, 256, 128, 128)),
    ("wg s2 P=8192 R512 Cg256", (32, 2, 16, 16, 32, 32, 512, 256, 256)),
    ("wg s2 P=2048 R512 Cg512", (32, 2, 8, 8, 16, 16, 512, 512, 512)),
]


def run_once(prob, force):
    B, s, dh, dw, gh, gw, R, Cg, Cg_out = prob
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    d = (torch.randn((B, dh, dw, R), device=dev, generator=g) * 0.5).to(torch.bfloat16)
    x = (torch.randn((B, gh, gw, Cg), device=dev, generator=g) * 0.5).to(torch.bfloat16)
    lib = L.lib()
    fp = (ctypes.c_int32 * 2)(*force)
    ws_b = ctypes.c_int64()
    assert lib.stc_conv_wgrad_query(L.BF16, B, dh, dw, R, Cg, fp, ctypes.byref(ws_b), None) == 0
    ws = torch.empty(max(int(ws_b.value), 16), dtype=torch.uint8, device=dev)
    dW = torch.empty((R, Cg_out, 4, 4), device=dev)
    rc = lib.stc_conv_wgrad_ex(L.BF16, B, s, L.nhwc_view(d), R, None, None, 0, 0.0, L.nhwc_view(x), Cg, Cg_out, None,
                               None, 0, 0.0, L.ptr(dW), fp, L.ptr(ws), int(ws_b.value), L.stream())
    assert rc == 0, lib.stc_last_error().decode()
    torch.cuda.synchronize()
    return dW


def main():
    for name, prob in PROBS:
        B, s, dh, dw, gh, gw, R, Cg, _ = prob
        fl = 2.0 * B * dh * dw * R * 16 * Cg
        ref = run_once(prob, (0, 16))
        line = f"{name:26s} auto {tune_wgrad.bench(prob, None, reps=20):7.1f} us"
        for c in (6, 7):
            same = torch.equal(ref.view(torch.int32), run_once(prob, (c, 16)).view(torch.int32))
            line += f" | cfg{c}/16 {'bit-identical' if same else 'DIFFERS'}"
            for ns in (0, 8, 16, 32):
                t = tune_wgrad.bench(prob, (c, ns), reps=20)
                if t is not None:
                    line += f" ns{ns} {t:6.1f} us {fl / t / 1e6:5.0f} TF"
        print(line, flush=True)


if __name__ == "__main__":
    main()
