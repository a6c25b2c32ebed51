"""Diagnostic: is the PatchGAN logits-layer weight gradient (stc_conv_wgrad_rows) deterministic under
load?  One process computes it ITERS times on identical inputs (the bench shape: B=32, 31x31x512 bf16
input, 30x30 gradient with one real channel) while a second stream keeps the GPU busy with large GEMMs
(--load), and counts results that differ bitwise from the first one.  Run it against the shipped library
(non-packed v_fma_f32 accumulations) and against the STC_ROWS_PACKED diagnostic build
(scripts/build_rows_packed.sh; the compiler's v_pk_fma_f32 form) via STC_LIB_PATH, alone or as two
concurrent processes (round 2's failure needed two processes on the GPU).

  python scripts/rows_stress.py --iters 400 --load [--tag name]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))

import torch  # noqa: E402

from stcgan_amd import _lib as L  # noqa: E402
from stcgan_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=400)
    ap.add_argument("--load", action="store_true")
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    B, C, H = 32, 512, 31
    x = (torch.rand((B, H, H, C), generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
    dy = torch.zeros((B, H - 1, H - 1, 8), device=dev)
    dy[..., 0] = torch.rand((B, H - 1, H - 1), generator=g, device=dev) * 2 - 1
    dy = dy.to(torch.bfloat16)
    # background load: the discriminator's 256->512 stride-1 conv (the bench's biggest GEMM shape)
    lx = (torch.rand((B, 32, 32, 256), generator=g, device=dev) * 2 - 1).to(torch.bfloat16)
    lw = (torch.rand((1, 512, 16, 256), generator=g, device=dev) * 0.02).to(torch.bfloat16)
    ly = torch.empty((B, 31, 31, 512), dtype=torch.bfloat16, device=dev)
    side = torch.cuda.Stream(dev)

    def rows():
        return ops.wgrad(B, 1, L.nhwc_view(dy), 8, L.nhwc_view(x), C, C, torch.bfloat16, device=dev, rows=1,
                         rows_kernel=True)

    ref = rows().clone()
    torch.cuda.synchronize()
    bad, first_bad = 0, None
    outs = []
    t0 = time.time()
    for i in range(a.iters):
        if a.load:
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(2):
                    ops.conv(L.CONV_S1, B, L.nhwc_view(lx), 256, lw, 512, L.nhwc_view(ly), torch.bfloat16)
        outs.append(rows())
        if len(outs) == 16 or i == a.iters - 1:
            torch.cuda.synchronize()
            for o in outs:
                d = (o != ref)
                if bool(d.any()):
                    bad += 1
                    if first_bad is None:
                        idx = d.nonzero()[:8].tolist()
                        first_bad = (idx, float((o - ref).abs().max()), float(ref.abs().max()))
            outs = []
    torch.cuda.synchronize()
    lib = os.path.basename(L.LIB_PATH)
    print(f"rows_stress[{a.tag}] lib={lib} load={a.load} iters={a.iters}: {bad} results differ from the first "
          f"({time.time() - t0:.1f} s){'' if first_bad is None else f'; first: idx {first_bad[0]} max {first_bad[1]:.3e} of {first_bad[2]:.3e}'}",
          flush=True)


if __name__ == "__main__":
    main()
