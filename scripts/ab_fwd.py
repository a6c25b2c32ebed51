"""A/B timer: one train-mode G1+G2 forward at bs=32 256x256 (bf16), HIP events over 20 reps.
Run once per configuration (environment-controlled tuning hooks) and compare the printed ms."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))

import torch  # noqa: E402

from stcgan_amd import networks  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    g1 = networks.get_generator(3, 1).apply(networks.weights_init).to(dev).set_compute_dtype("bf16").train()
    g2 = networks.get_generator(4, 3).apply(networks.weights_init).to(dev).set_compute_dtype("bf16").train()
    x = torch.rand((32, 3, 256, 256), device=dev) * 2 - 1
    with torch.no_grad():
        for _ in range(3):
            m = g1(x)
            y = g2([x, m])
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            m = g1(x)
            y = g2([x, m])
        e1.record()
        e1.synchronize()
    print(f"{os.environ.get('AB_TAG', '')} g1g2 fwd {e0.elapsed_time(e1) / 20:.3f} ms  "
          f"chk {float(m.float().abs().mean()):.6f} {float(y.float().abs().mean()):.6f}")


if __name__ == "__main__":
    main()
