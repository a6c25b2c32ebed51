"""Diagnostic for G2 deep-level gradient mismatch: determinism and variants (prints only)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "shadow-removal-istd_amd"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
from fixture_init import fixture_state, normal, uniform  # noqa: E402
from oracle import stcgan_ref as ref  # noqa: E402
from stcgan_amd import networks  # noqa: E402


def run(in_c, out_c, seed, bs=2, hw=256, ngf=8):
    net = networks.get_generator(in_c, out_c, ngf=ngf)
    st = fixture_state(net.state_dict(), seed, "one")
    net.load_state_dict(st)
    net.cuda().train()
    x = uniform((bs, in_c, hw, hw), 100 + seed)
    xg = x.cuda().requires_grad_(True)
    out = net(xg)
    r = normal(tuple(out.shape), 200 + seed)
    (out * r.cuda()).sum().backward()
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().cpu().clone() for k, p in net.named_parameters()}
    # oracle
    pr = {k: v.clone().requires_grad_(not ref._is_buffer(k) and v.is_floating_point()) for k, v in st.items()}
    xo = x.clone().requires_grad_(True)
    oo = ref.generator_forward(pr, xo, True)
    (oo * r).sum().backward()
    worst = []
    for k in grads:
        e = float((grads[k] - pr[k].grad).abs().max() / (pr[k].grad.abs().max() + 1e-30))
        worst.append((e, k))
    worst.sort(reverse=True)
    ein = float((xg.grad.cpu() - xo.grad).abs().max() / xo.grad.abs().max())
    return grads, worst[:4], ein


for (in_c, out_c, seed, bs) in [(4, 3, 12, 2), (4, 3, 12, 2), (3, 1, 11, 2), (4, 3, 11, 2), (3, 3, 12, 2),
                                (4, 1, 12, 2), (4, 3, 12, 1), (4, 3, 12, 4)]:
    g, worst, ein = run(in_c, out_c, seed, bs)
    print(f"in={in_c} out={out_c} seed={seed} bs={bs}: input-grad rel {ein:.2e}; worst param rel "
          + ", ".join(f"{e:.1e}:{k[-22:]}" for e, k in worst), flush=True)
g1, _, _ = run(4, 3, 12)
g2, _, _ = run(4, 3, 12)
diff = max(float((g1[k] - g2[k]).abs().max()) for k in g1)
print("run-to-run max grad diff (same inputs):", diff)
