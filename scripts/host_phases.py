"""Host-side time of each phase of the bf16 bs=32 train step (no syncs added): where does the host
fall behind the GPU?  Wraps backward(), the optimiser steps, network calls and the losses."""
import collections
import os
import sys
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shadow-removal-istd_amd"))
import torch  # noqa: E402

from stcgan_amd import engine, loss, optim  # noqa: E402
from stcgan_amd.stcgan import STCGAN  # noqa: E402

acc = collections.defaultdict(float)
cnt = collections.Counter()


def wrap(obj, name, tag):
    f = getattr(obj, name)

    def g(*a, **k):
        t = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            acc[tag] += time.perf_counter() - t
            cnt[tag] += 1
    setattr(obj, name, g)


wrap(torch.Tensor, "backward", "backward")
wrap(optim.Adam, "step", "adam")
wrap(engine.NetFn, "apply", "net fwd")
wrap(loss._LossFn, "apply", "loss fwd")
a = types.SimpleNamespace(devices=["cuda:0"], tasks=["train"], lr_G=5e-5, lr_D=2e-5, beta1=0.5, beta2=0.999,
                          D_loss_fn="standard", D_loss_type="normal", ngf=64, dtype="bf16", load_weights_g1=None,
                          load_weights_g2=None, load_weights_d1=None, load_weights_d2=None)
tr = STCGAN(a)
dev = torch.device("cuda", 0)
x = torch.rand((32, 3, 256, 256), device=dev) * 2 - 1
m = (torch.rand((32, 1, 256, 256), device=dev) < 0.5).float() * 2 - 1
y = torch.rand((32, 3, 256, 256), device=dev) * 2 - 1
for _ in range(3):
    tr.train_step(x, m, y)
torch.cuda.synchronize()
acc.clear()
cnt.clear()
N = 10
t0 = time.perf_counter()
for _ in range(N):
    t = time.perf_counter()
    tr.train_step(x, m, y)
    acc["train_step (host)"] += time.perf_counter() - t
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / N
print(f"wall {wall * 1e3:.3f} ms/step", flush=True)
for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
    print(f"{v / N * 1e3:8.3f} ms/step  {cnt[k] / N:5.1f} calls  {k}", flush=True)

# which optimiser path runs, and how long the table upload takes
stats = collections.Counter()
fast0 = optim.Adam._fast_step


def fast(self, gi, group):
    r = fast0(self, gi, group)
    stats["fast" if r else "slow"] += 1
    return r


optim.Adam._fast_step = fast
orig_tensor = torch.tensor
for _ in range(5):
    tr.train_step(x, m, y)
torch.cuda.synchronize()
print("optimizer group paths over 5 steps:", dict(stats), flush=True)
for o in (tr.optim_D, tr.optim_G):
    f = o._fast.get(0)
    print("fast record:", None if f is None else (len(f["plist"]), f["step"], f["epoch"]), "epoch now",
          __import__("stcgan_amd.ops", fromlist=["x"]).PACK_EPOCH, flush=True)
