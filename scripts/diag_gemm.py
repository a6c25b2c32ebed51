"""What the parts of a bf16 GEMM tile cost: times a fixed set of conv-forward and weight-gradient
problems of the bs=32 train step (auto plans, kernel + any split reduction, HIP-graph replay) with
whichever library STC_LIB_PATH names -- run once per diagnostic variant of scripts/diag_gemm.sh
(no DMA / no MFMA / no epilogue) and compare with the shipped library.  Prints one line per problem."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import tune_bf16  # noqa: E402
import tune_wgrad  # noqa: E402
from stcgan_amd import _lib as L  # noqa: E402

B = 32
CONV = [  # (kind, B, gh, gw, xh, xw, yh, yw, cin, cout)
    ("e2 conv_s2 64x64 64->128", (L.CONV_S2, B, 64, 64, 128, 128, 64, 64, 64, 128)),
    ("e3 conv_s2 32x32 128->256", (L.CONV_S2, B, 32, 32, 64, 64, 32, 32, 128, 256)),
    ("e4 conv_s2 16x16 256->512", (L.CONV_S2, B, 16, 16, 32, 32, 16, 16, 256, 512)),
    ("d4 convT 16x16 1024->256", (L.CONVT_S2, B, 16, 16, 16, 16, 32, 32, 1024, 256)),
    ("d3 convT 32x32 512->128", (L.CONVT_S2, B, 32, 32, 32, 32, 64, 64, 512, 128)),
    ("d2 convT 64x64 256->64", (L.CONVT_S2, B, 64, 64, 64, 64, 128, 128, 256, 64)),
    ("D4 conv_s1 31x31 256->512", (L.CONV_S1, B, 31, 31, 32, 32, 31, 31, 256, 512)),
]
WGRAD = [  # (B, s, dh, dw, gh, gw, R, Cg, Cg_out)
    ("wg s2 P=131072 R128 Cg64", (B, 2, 64, 64, 128, 128, 128, 64, 64)),
    ("wg s2 P=32768 R256 Cg128", (B, 2, 32, 32, 64, 64, 256, 128, 128)),
    ("wg s1 P=30752 R512 Cg256", (B, 1, 31, 31, 32, 32, 512, 256, 256)),
]


def main():
    tag = os.path.basename(os.environ.get("STC_LIB_PATH") or "shipped")
    for name, prob in CONV:
        kind, b, gh, gw, xh, xw, yh, yw, cin, cout = prob
        taps, nph = (4, 4) if kind == L.CONVT_S2 else (16, 1)
        fl = 2.0 * b * gh * gw * nph * cout * taps * cin
        t = tune_bf16.bench(prob, None, reps=20)
        print(f"{tag:16s} {name:28s} {t:8.1f} us {fl / t / 1e6:7.1f} TF", flush=True)
    for name, prob in WGRAD:
        b, s, dh, dw, gh, gw, R, Cg, _ = prob
        fl = 2.0 * b * dh * dw * R * 16 * Cg
        t = tune_wgrad.bench(prob, None, reps=20)
        print(f"{tag:16s} {name:28s} {t:8.1f} us {fl / t / 1e6:7.1f} TF", flush=True)


if __name__ == "__main__":
    main()
