"""Interleaved A/B of forced conv plans in the north-star G1+G2 bf16 forward (bs 32, 256x256, train-mode BN): each
variant sets ops.FORCE_CONV (keyed (kind, B, gh, gw, cin, cout) -> (tile config, splits)), the forward is captured as
a HIP graph and replayed; rounds alternate the variants, the median per variant is printed.

  python scripts/ab_force_fwd.py
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))

import torch  # noqa: E402

from stcgan_amd import _lib as L  # noqa: E402
from stcgan_amd import networks, ops  # noqa: E402

B = 32
E5 = {(L.CONV_S2, B, 8, 8, 512, 512): (5, 4)}
E6 = {(L.CONV_S2, B, 4, 4, 512, 512): (12, 4)}
D7 = {(L.CONVT_S2, B, 2, 2, 1024, 512): (12, 4)}
D8 = {(L.CONVT_S2, B, 1, 1, 512, 512): (12, 4)}
VARIANTS = {  # name -> FORCE_CONV
    "auto": {},
    "e5": E5,
    "e6": E6,
    "e5+e6": {**E5, **E6},
    "e5+e6+d7": {**E5, **E6, **D7},
    "e5+e6+d7+d8": {**E5, **E6, **D7, **D8},
}


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    g1 = networks.get_generator(3, 1).apply(networks.weights_init).to(dev).set_compute_dtype("bf16").train()
    g2 = networks.get_generator(4, 3).apply(networks.weights_init).to(dev).set_compute_dtype("bf16").train()
    x = torch.rand((B, 3, 256, 256), device=dev) * 2 - 1

    def fwd():
        m = g1(x)
        return g2([x, m])

    graphs = {}
    with torch.no_grad():
        for name, force in VARIANTS.items():
            ops.FORCE_CONV.clear()
            ops.FORCE_CONV.update(force)
            for _ in range(2):
                fwd()
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            st = torch.cuda.Stream()
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st):
                with torch.cuda.graph(gr, stream=st):
                    fwd()
            torch.cuda.synchronize()
            graphs[name] = gr
        ops.FORCE_CONV.clear()
        times = {k: [] for k in graphs}
        for _ in range(7):
            for name, gr in graphs.items():
                gr.replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    gr.replay()
                e1.record()
                e1.synchronize()
                times[name].append(e0.elapsed_time(e1) / 3)
    for name, ts in times.items():
        print(f"{name:14s} median {statistics.median(ts):.4f} ms  (min {min(ts):.4f})", flush=True)


if __name__ == "__main__":
    main()
