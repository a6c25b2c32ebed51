"""One G1+G2 train-mode forward at bs=32 256x256 (the north-star kernel set), after two
warm-up forwards: the program rocprofv3 --pmc passes run to measure HBM traffic per launch
of the dominant implicit-GEMM kernel (scripts/pmc_traffic.py reads the counters)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))

import torch  # noqa: E402

from stcgan_amd import networks  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--reps", type=int, default=1)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    g1 = networks.get_generator(3, 1).apply(networks.weights_init).to(dev).set_compute_dtype(a.dtype).train()
    g2 = networks.get_generator(4, 3).apply(networks.weights_init).to(dev).set_compute_dtype(a.dtype).train()
    x = torch.rand((a.batch, 3, a.size, a.size), device=dev) * 2 - 1
    with torch.no_grad():
        for _ in range(2 + a.reps):
            m = g1(x)
            g2([x, m])
    torch.cuda.synchronize()
    print("done", float(m.float().abs().mean()))


if __name__ == "__main__":
    main()
