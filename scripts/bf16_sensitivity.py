"""How chaotic is the ST-CGAN gradient in bf16 storage?  Runs the oracle's bf16 mode (oracle/stcgan_ref.py
Precision: the HIP bf16 path's storage points) twice on the same batch -- once from the reference-init
weights, once with every parameter scaled by (1 + 1e-6 N(0,1)), the size of an accumulation-order
difference -- and prints the per-tensor relative L2 of the resulting gradients, in module order.
Round 3 (ngf=64, bs=4..32, G1+G2 with the L1 data losses): bf16 median 13 %, worst 20 % (the innermost
levels; the error grows through each BatchNorm backward); fp32 0.3 %.  This is the noise floor a
whole-step bf16 comparison sits on (tests/test_gpu_configs.py), which is why the discriminating bf16
check is per layer (tests/test_gpu_c3_layers.py).

  python scripts/bf16_sensitivity.py [bf16|fp32] [batch] [ref|one]
"""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]

import torch  # noqa: E402

from fixture_init import fixture_state, pm_one, uniform  # noqa: E402
from oracle import stcgan_ref as ref  # noqa: E402


def main():
    prec = ref.FP32 if (len(sys.argv) > 1 and sys.argv[1] == "fp32") else ref.BF16
    bs = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    fam = sys.argv[3] if len(sys.argv) > 3 else "ref"
    torch.set_num_threads(os.cpu_count() or 8)
    ngf = 64
    st = {"G1": fixture_state(ref.generator_state_template(3, 1, ngf), 11, fam),
          "G2": fixture_state(ref.generator_state_template(4, 3, ngf), 12, fam)}
    x, m, y = uniform((bs, 3, 256, 256), 8100), pm_one((bs, 1, 256, 256), 8101), uniform((bs, 3, 256, 256), 8102)

    def run(eps):
        s = copy.deepcopy(st)
        g = torch.Generator().manual_seed(1)
        for n in s:
            for k, v in s[n].items():
                if v.is_floating_point() and not ref._is_buffer(k):
                    v.mul_(1 + eps * torch.randn(v.shape, generator=g))
                    v.requires_grad_(True)
        mp = ref.generator_forward(s["G1"], x, True, prec=prec)
        yp = ref.generator_forward(s["G2"], torch.cat((x, mp), 1), True, prec=prec)
        (ref.data_loss(mp, m) + 5 * ref.data_loss(yp, y)).backward()
        return s

    a, c = run(0.0), run(1e-6)
    for n in ("G1", "G2"):
        rows = []
        for k, v in a[n].items():
            if v.is_floating_point() and not ref._is_buffer(k):
                rows.append((float((v.grad - c[n][k].grad).norm() / (c[n][k].grad.norm() + 1e-30)), k))
        errs = sorted(e for e, _ in rows)
        print(f"{n} ({'bf16' if prec.bf16 else 'fp32'}, bs={bs}, {fam}): median {errs[len(errs) // 2]:.4f}, "
              f"worst {errs[-1]:.4f}")
        for e, k in rows:
            print(f"  {e:.4f} {k}")


if __name__ == "__main__":
    main()
