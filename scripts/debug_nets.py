"""Diagnostic: per-tensor errors of the HIP networks vs the ngf=8 goldens (prints, never asserts)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "shadow-removal-istd_amd"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
from fixture_init import fixture_state, normal, uniform  # noqa: E402
from stcgan_amd import networks  # noqa: E402

NET_IN = {"G1": 3, "G2": 4, "D1": 4, "D2": 7}
NET_SEED = {"G1": 11, "G2": 12, "D1": 13, "D2": 14}
d = dict(np.load(os.path.join(ROOT, "tests", "golden", "nets_ngf8.npz")))


def rel(key, t):
    t = t.detach().cpu().double()
    if key in d:
        r = torch.from_numpy(d[key]).double()
        return float((t - r).abs().max()), float(r.abs().max())
    idx = torch.from_numpy(d[key + "::idx"])
    r = torch.from_numpy(d[key + "::val"]).double()
    return float((t.reshape(-1)[idx] - r).abs().max()), float(r.abs().max())


for name in sys.argv[1:] or ["G1", "G2"]:
    if name.startswith("G"):
        net = networks.get_generator(NET_IN[name], 1 if name == "G1" else 3, ngf=8)
    else:
        net = networks.get_discriminator(NET_IN[name], ndf=8)
    net.load_state_dict(fixture_state(net.state_dict(), NET_SEED[name], "one"))
    net.cuda().train()
    x = uniform((2, NET_IN[name], 256, 256), 100 + NET_SEED[name]).cuda().requires_grad_(True)
    out = net(x)
    r = normal(tuple(out.shape), 200 + NET_SEED[name]).cuda()
    (out * r).sum().backward()
    torch.cuda.synchronize()
    e, s = rel(f"{name}/train_out", out)
    print(f"{name} out err {e:.3e} scale {s:.3e}")
    e, s = rel(f"{name}/input_grad", x.grad)
    print(f"{name} input_grad err {e:.3e} scale {s:.3e}")
    if name == "G2":
        g = x.grad.detach().cpu()
        ref_full = None
        for c in range(4):
            print("  channel", c, "absmax", float(g[:, c].abs().max()))
    for k, p in net.named_parameters():
        e, s = rel(f"{name}/grad/{k}", p.grad)
        print(f"  {k:60s} err {e:.3e} scale {s:.3e} rel {e / (s + 1e-30):.2e}")
